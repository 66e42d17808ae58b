set -o pipefail
bash scripts/gpu_step.sh zd_tests 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c2.py tests/test_gpu_unet.py -x -q --timeout 300 --timeout-method thread -rf -k "groupnorm or gn or c2 or fused or teacher" || exit 99
bash scripts/gpu_step.sh zd_ab_fq 500 bash scripts/ab_env.sh QD_NO_GN_FIN_SMALL=1 2 --no-e2e || exit 99
