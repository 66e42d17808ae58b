set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 --timeout-method thread -rf tests -m gpu -k "attn or attention or absmax or colmax or act_quant or per_channel" > gpurun_out/r05zf_tests.log 2>&1 || exit 11
tail -2 gpurun_out/r05zf_tests.log
timeout -k 10 120 python3 scripts/attn_bench.py > gpurun_out/r05zf_attn0.log 2>&1 || exit 12
timeout -k 10 120 python3 scripts/attn_bench.py 6 > gpurun_out/r05zf_attn6.log 2>&1 || exit 13
head -2 gpurun_out/r05zf_attn0.log gpurun_out/r05zf_attn6.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05zf_smoke.log 2>&1 || exit 14
tail -1 gpurun_out/r05zf_smoke.log
