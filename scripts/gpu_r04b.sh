# GroupNorm statistics in the int8 producing epilogues: tests, incremental table tune, A/B, profile
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04b_tests 700 python -u -m pytest tests/test_gpu_int8.py tests/test_calib_mean.py \
  "tests/test_gpu_kernels.py::test_attention_sharp_softmax" -x -q --timeout 300 --timeout-method thread -rf || exit 99
bash scripts/gpu_step.sh r04b_tune 300 python -u scripts/tune_table.py --add --models sd15 --out gpurun_out/gemm_table.json || exit 99
export QD_GEMM_TABLE=$PWD/gpurun_out/gemm_table.json
bash scripts/gpu_step.sh r04b_ab_gnpart 600 bash scripts/ab_env.sh QD_NO_GN_PART=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
bash scripts/prof_bench.sh r04b_int8 400 --mode w8a8-sq-int8 --no-e2e || exit 99
