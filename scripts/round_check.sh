# full GPU check of the tree: parity suite, smoke, the three bench lines, rocprof of the headline bench
# (test failures (pytest rc 1) are recorded and the check goes on; a crash, abort or time limit ends it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/rc_tests.log 2>&1
rc=$?
echo "[rc] tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rc_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/rc_bench_sd15.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --mode w8a8-sq-int8 > gpurun_out/rc_bench_int8.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --model sdxl --steps 2 > gpurun_out/rc_bench_sdxl.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --model sd35 --denoise-steps 10 --steps 2 > gpurun_out/rc_bench_sd35.log 2>&1 || exit 1
bash scripts/prof_bench.sh rc 300 || exit 1
exit $rc
