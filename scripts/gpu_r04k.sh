# M-fastest block order for weight-heavy GEMMs / convs + conflict-free k_attn32 K rows:
# kernel tests, attention A/B, conv timings and bench A/Bs of QD_NO_MFAST
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04k_tests 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_int8.py -x -q --timeout 300 --timeout-method thread -rf || exit 99
grep -q " passed" gpurun_out/r04k_tests.log && ! grep -q "failed" gpurun_out/r04k_tests.log || exit 98
bash scripts/gpu_step.sh r04k_attn_old 120 env QD_ATTN_CFG=6 python -u scripts/attn_bench.py || exit 99
bash scripts/gpu_step.sh r04k_attn_new 120 python -u scripts/attn_bench.py || exit 99
bash scripts/gpu_step.sh r04k_conv_nomfast 200 env QD_NO_MFAST=1 python -u scripts/i8_bench.py || exit 99
bash scripts/gpu_step.sh r04k_conv_mfast 200 python -u scripts/i8_bench.py || exit 99
bash scripts/gpu_step.sh r04k_ab_fq 600 bash scripts/ab_env.sh QD_NO_MFAST=1 2 || exit 99
bash scripts/gpu_step.sh r04k_ab_int8 600 bash scripts/ab_env.sh QD_NO_MFAST=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
