#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench run (writes gpurun_out/prof_<tag>/...); the raw
# kernel trace is reduced on the box to the per-eval summary, the step classes and the step's
# launch sequence, then deleted (it is larger than what gpurun copies back)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_${1:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${2:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-int8-mode "${@:3}" > "$OUT/bench.log" 2>&1
rc=$?
echo "[prof] rc=$rc"
tail -3 "$OUT/bench.log"
TR=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
if [ -n "$TR" ]; then
  python3 "$ROOT/scripts/prof_summary.py" "$TR" > "$OUT/per_eval.txt" 2>&1
  python3 "$ROOT/scripts/step_classes.py" "$TR" > "$OUT/step_classes.txt" 2>&1
  python3 "$ROOT/scripts/eval_sequence.py" "$TR" > "$OUT/step_sequence.txt" 2>&1
  rm -f "$TR"
fi
find "$OUT" -name "*.csv" -size +8M -delete
find "$OUT" -name "*kernel_stats.csv" | head -3
exit $rc
