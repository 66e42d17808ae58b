# k_attn32 generalized to head_dim 64 / 80: attention tests, A/B vs the 16x16x32 kernel, PMC
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04n_attn_tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k attention --timeout 120 --timeout-method thread -rf || exit 99
grep -q " passed" gpurun_out/r04n_attn_tests.log && ! grep -q "failed" gpurun_out/r04n_attn_tests.log || exit 98
bash scripts/gpu_step.sh r04n_attn_old 120 env QD_ATTN_CFG=6 python -u scripts/attn_bench.py || exit 99
bash scripts/gpu_step.sh r04n_attn_new 120 python -u scripts/attn_bench.py || exit 99
bash scripts/gpu_step.sh r04n_attn_new4 120 env QD_ATTN_CFG=7 python -u scripts/attn_bench.py || exit 99
bash scripts/gpu_step.sh r04n_attn_new8 120 env QD_ATTN_CFG=8 python -u scripts/attn_bench.py || exit 99
