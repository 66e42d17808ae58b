set -o pipefail
bash scripts/gpu_step.sh bench_r03e 400 python -u bench.py --no-cpu-baseline || exit 99
bash scripts/gpu_step.sh bench_r03e_int8 400 python -u bench.py --no-cpu-baseline --no-e2e --mode w8a8-sq-int8 || exit 99
bash scripts/prof_bench.sh r03e_int8 400 --mode w8a8-sq-int8 --no-e2e || exit 99
