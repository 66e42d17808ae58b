# full GPU check (part 2): the secondary bench lines and rocprof profiles of the final tree
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh y_bench_sdxl 300 python -u bench.py --model sdxl --steps 2 --no-cpu-baseline || exit 99
bash scripts/gpu_step.sh y_bench_sd35 300 python -u bench.py --model sd35 --denoise-steps 10 --steps 2 --no-cpu-baseline || exit 99
bash scripts/prof_bench.sh r03y 400 || exit 99
bash scripts/prof_bench.sh r03y_int8 400 --mode w8a8-sq-int8 --no-e2e || exit 99
