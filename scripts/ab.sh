#!/bin/bash
# A/B: bench.py with scripts/ab/libqdiff_prev.so vs the in-tree build, alternating on ONE box
# (box-to-box clock differences are larger than most single-change effects).
# usage: bash scripts/ab.sh <rounds> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=${1:-2}; shift
for i in $(seq 1 "$R"); do
  for lib in prev new; do
    if [ "$lib" = prev ]; then export QD_LIB_PATH=$ROOT/scripts/ab/libqdiff_prev.so; else unset QD_LIB_PATH; fi
    out=$(timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "[ab] $lib failed"; exit 1; }
    echo "[ab] round $i $lib: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
