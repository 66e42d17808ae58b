# attention configuration sweep (QD_ATTN_CFG read once per process)
set -e
for c in 0 1 2 3 5; do
  if [ $c = 0 ]; then unset QD_ATTN_CFG; else export QD_ATTN_CFG=$c; fi
  timeout -k 10 60 python3 scripts/attn_bench.py 2>/dev/null
done
