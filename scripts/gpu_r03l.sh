set -o pipefail
bash scripts/gpu_step.sh gn_i8_tests 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread -k "groupnorm or gn_ or fin or int8 or i8" || exit 99
QD_NO_I8_AMAX_FUSE=1 bash scripts/gpu_step.sh ab_gn_int8 600 bash scripts/ab.sh 2 --mode w8a8-sq-int8 --no-e2e || exit 99
bash scripts/gpu_step.sh ab_fuse_int8 600 bash scripts/ab_env.sh QD_NO_I8_AMAX_FUSE=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
