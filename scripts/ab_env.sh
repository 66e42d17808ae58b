#!/bin/bash
# A/B of one environment switch on ONE box: bench.py with VAR=VALUE ("prev") vs without ("new"), alternating.
# usage: bash scripts/ab_env.sh VAR=VALUE <rounds> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
KV=$1; shift
R=${1:-2}; shift
for i in $(seq 1 "$R"); do
  for side in prev new; do
    if [ "$side" = prev ]; then out=$(env "$KV" timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }
    else out=$(timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }; fi
    echo "[ab] round $i $side: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "int8_mode", (d.get("int8_mode") or {}).get("value"))')"
  done
done
