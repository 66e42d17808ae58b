# final GPU check of the round-3 tree (short form): parity suite, smoke, headline + int8 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/zf_tests.log 2>&1
rc=$?
echo "[zf] tests rc=$rc"; tail -3 gpurun_out/zf_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/zf_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/zf_smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/zf_bench_sd15.log 2>&1 || exit 1
tail -1 gpurun_out/zf_bench_sd15.log | cut -c1-300
bash scripts/gpu_step.sh zf_bench_int8 300 python -u bench.py --mode w8a8-sq-int8 --no-cpu-baseline --no-e2e || exit 99
exit $rc
