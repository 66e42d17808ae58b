#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench run (writes gpurun_out/prof/...)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_${1:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${2:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline "${@:3}" > "$OUT/bench.log" 2>&1
rc=$?
echo "[prof] rc=$rc"
tail -3 "$OUT/bench.log"
find "$OUT" -name "*kernel_stats.csv" | head -3
exit $rc
