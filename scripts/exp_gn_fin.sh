# GroupNorm-fin (residual and temb forms): kernel tests, model tests, same-box A/B (prev = QD_NO_GN_FIN=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_int8.py -m gpu -q --timeout 120 --timeout-method thread -rf -k "groupnorm" > gpurun_out/x_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_unet.py tests/test_gpu_configs.py tests/test_gpu_sdxl.py tests/test_gpu_dist.py -m gpu -q --timeout 200 --timeout-method thread -rf > gpurun_out/x_tests2.log 2>&1; rc=$?; echo "tests2 rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 scripts/mem_bench.py > gpurun_out/x_mem.log 2>&1 || exit 3
timeout -k 10 900 bash scripts/ab_env.sh QD_NO_GN_FIN=1 2 --steps 3 > gpurun_out/x_ab.log 2>&1 || exit 4
