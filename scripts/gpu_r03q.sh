set -o pipefail
bash scripts/gpu_step.sh q_tests 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread -k "post_residual or amax or linear" || exit 99
bash scripts/gpu_step.sh q_ab 600 bash scripts/ab.sh 3 --no-e2e || exit 99
