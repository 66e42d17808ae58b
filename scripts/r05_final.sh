#!/bin/bash
# round-5 final measurements (after the full GPU suite ran in its own call): smoke, the default bench
# line (fake-quant headline + int8_mode object), rocprof step profiles of both modes
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r05z}
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 11
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit 12
tail -c 1500 gpurun_out/${TAG}_bench.log
timeout -k 10 450 bash scripts/prof_bench.sh ${TAG}_fq 400 > gpurun_out/${TAG}_prof_fq.log 2>&1 || exit 13
timeout -k 10 450 bash scripts/prof_bench.sh ${TAG}_int8 400 --mode w8a8-sq-int8 > gpurun_out/${TAG}_prof_int8.log 2>&1 || exit 14
head -14 gpurun_out/prof_${TAG}_fq/step_classes.txt gpurun_out/prof_${TAG}_int8/step_classes.txt
