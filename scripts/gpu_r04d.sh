# concat GroupNorm from two producers' slot statistics + packed slot statistics: tests, re-tune, A/B, profile
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04d_tests 700 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 300 --timeout-method thread -rf || exit 99
bash scripts/gpu_step.sh r04d_tune 300 python -u scripts/tune_table.py --add --drop-epi 384 --models sd15 --out gpurun_out/gemm_table.json || exit 99
export QD_GEMM_TABLE=$PWD/gpurun_out/gemm_table.json
bash scripts/gpu_step.sh r04d_ab_gnpart 600 bash scripts/ab_env.sh QD_NO_GN_PART=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
bash scripts/prof_bench.sh r04d_int8 400 --mode w8a8-sq-int8 --no-e2e || exit 99
