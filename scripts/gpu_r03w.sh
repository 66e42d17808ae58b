set -o pipefail
bash scripts/gpu_step.sh w_gn_sweep 300 python -u scripts/gn_bench.py --sweep || exit 99
