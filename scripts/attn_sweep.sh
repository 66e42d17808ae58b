# attention configuration sweep (qd_attn_force, one process per setting)
set -e
for c in 0 1 2 3 5; do
  timeout -k 10 60 python3 scripts/attn_bench.py $c 2>/dev/null
done
