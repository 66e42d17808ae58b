# direct-store epilogue: bit-equality test, then the short-K / GEGLU microbenchmarks under both forms
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r05e}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_epilogue.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_epi_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_epi_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u scripts/epi_ab.py > gpurun_out/${TAG}_epi_ab.log 2>&1 || exit 1
cat gpurun_out/${TAG}_epi_ab.log
exit $rc
