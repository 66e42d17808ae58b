#!/bin/bash
# HBM traffic of the dominant kernel: two separate --pmc passes (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/pmc_${1:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$ROOT/scripts/roof_kernel.py" 10 > "$OUT/fetch.log" 2>&1 || exit 99
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$ROOT/scripts/roof_kernel.py" 10 > "$OUT/write.log" 2>&1 || exit 99
echo "[pmc] done"; find "$OUT" -name "*counter_collection.csv"
