set -o pipefail
bash scripts/gpu_step.sh s_tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_int8.py tests/test_gpu_c2.py -x -q --timeout 300 --timeout-method thread -rf -k "layernorm or c2" || exit 99
bash scripts/gpu_step.sh s_ab_fq 600 bash scripts/ab_env.sh QD_LN_ROWS_OFF=1 2 --no-e2e || exit 99
bash scripts/gpu_step.sh s_ab_int8 600 bash scripts/ab_env.sh QD_LN_ROWS_OFF=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
