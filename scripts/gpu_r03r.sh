set -o pipefail
bash scripts/gpu_step.sh r_tests 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_c2.py tests/test_gpu_determinism.py tests/test_gpu_sdxl.py -x -q --timeout 300 --timeout-method thread -rf || exit 99
bash scripts/gpu_step.sh r_ab_fq 600 bash scripts/ab_env.sh QD_NO_SIDE_STREAM=1 2 --no-e2e || exit 99
bash scripts/gpu_step.sh r_ab_int8 600 bash scripts/ab_env.sh QD_NO_SIDE_STREAM=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
