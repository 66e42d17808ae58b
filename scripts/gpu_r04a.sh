# round 4 first box: PMC traffic of the fp16 / int8 halo convs, baseline benches of both modes
set -o pipefail
mkdir -p gpurun_out
bash scripts/pmc_traffic.sh r04a 202 142 || exit 99
bash scripts/gpu_step.sh r04a_bench_sd15 300 python -u bench.py --no-cpu-baseline --no-e2e || exit 99
bash scripts/gpu_step.sh r04a_bench_int8 300 python -u bench.py --mode w8a8-sq-int8 --no-cpu-baseline --no-e2e || exit 99
