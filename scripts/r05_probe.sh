# microbenchmarks of the int8 short-K / GEGLU GEMMs + profile of one int8 eval
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r05b}
timeout -k 10 300 python3 -u scripts/shortk_i8.py > gpurun_out/${TAG}_shortk.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/geglu_sweep.py > gpurun_out/${TAG}_geglu.log 2>&1 || exit 1
bash scripts/prof_bench.sh ${TAG}_int8 300 --mode w8a8-sq-int8 || exit 1
