#!/bin/bash
# A/B of a library + GEMM table pair: scripts/ab/libqdiff_prev.so with the committed table vs the
# in-tree build with the table in $NEW_TABLE, alternating on ONE box.
# usage: NEW_TABLE=<path> bash scripts/ab_table.sh <rounds> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=${1:-2}; shift
for i in $(seq 1 "$R"); do
  for lib in prev new; do
    if [ "$lib" = prev ]; then export QD_LIB_PATH=$ROOT/scripts/ab/libqdiff_prev.so; unset QD_GEMM_TABLE
    else unset QD_LIB_PATH; export QD_GEMM_TABLE=$NEW_TABLE; fi
    out=$(timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline --no-e2e "$@" 2>/dev/null | tail -1) || { echo "[ab] $lib failed"; exit 1; }
    echo "[ab] round $i $lib: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
