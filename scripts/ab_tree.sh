#!/bin/bash
# Same-box A/B of two whole trees (package + library + bench.py): ab_r05/ (the round-5 tree, built
# in-tree) vs this tree, alternating rounds on ONE box; prints the headline and int8_mode values.
# usage: bash scripts/ab_tree.sh <rounds> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=${1:-2}; shift
for i in $(seq 1 "$R"); do
  for side in r05 new; do
    dir=$ROOT; [ "$side" = r05 ] && dir=$ROOT/ab_r05
    out=$(cd "$dir" && timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --no-e2e "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }
    echo "[ab] round $i $side: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); i=d.get("int8_mode") or {}; print(d["value"], d["ms_per_step"], "int8_mode", i.get("value"), i.get("ms_per_step"))')"
  done
done
