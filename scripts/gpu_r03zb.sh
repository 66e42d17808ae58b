set -o pipefail
bash scripts/gpu_step.sh zb_tests 300 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread -rf -k "sample or conv or quant" || exit 99
bash scripts/gpu_step.sh zb_ab_int8 500 bash scripts/ab.sh 2 --mode w8a8-sq-int8 --no-e2e || exit 99
