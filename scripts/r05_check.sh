# round-5 check: GPU parity suite, smoke, default bench line (with the int8_mode object)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r05}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "[rc] tests rc=$rc"; tail -5 gpurun_out/${TAG}_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
tail -c 3000 gpurun_out/${TAG}_bench.log
exit $rc
