# one-off GPU experiment runner: self-test, attention tests + timings, same-box bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -m gpu -q --timeout 120 --timeout-method thread -rf -k "reciprocal or attention or attn or unet or layer" > gpurun_out/x_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 60 python3 scripts/attn_bench.py > gpurun_out/x_attn.log 2>&1 || exit 3
timeout -k 10 900 bash scripts/ab.sh 2 --steps 3 > gpurun_out/x_ab.log 2>&1 || exit 4
