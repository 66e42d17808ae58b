#!/bin/bash
# Same-box A/B of one bench.py flag: bench with FLAG ("prev") vs without ("new"), alternating rounds.
# usage: bash scripts/ab_flag.sh FLAG <rounds> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
FLAG=$1; shift
R=${1:-2}; shift
for i in $(seq 1 "$R"); do
  for side in prev new; do
    if [ "$side" = prev ]; then out=$(timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline --no-e2e --no-int8-mode "$FLAG" "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }
    else out=$(timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline --no-e2e --no-int8-mode "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }; fi
    echo "[ab] round $i $side: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
