set -o pipefail
bash scripts/gpu_step.sh za_tests 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c2.py -x -q --timeout 120 --timeout-method thread -rf -k "finalize or apply or act or fq or c2" || exit 99
bash scripts/gpu_step.sh za_ab_fq 500 bash scripts/ab.sh 2 --no-e2e || exit 99
