#!/bin/bash
# HBM traffic of the dominant conv per GEMM variant: separate --pmc passes (FETCH_SIZE, WRITE_SIZE)
# usage: scripts/pmc_dominant.sh TAG "100 200"
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/pmc_${1:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${2:-100}; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$v" -o run -- python3 "$ROOT/scripts/roof_kernel.py" 10 $v > "$OUT/fetch_$v.log" 2>&1 || exit 99
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$v" -o run -- python3 "$ROOT/scripts/roof_kernel.py" 10 $v > "$OUT/write_$v.log" 2>&1 || exit 99
done
echo "[pmc] done"
