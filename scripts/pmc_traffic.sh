#!/bin/bash
# HBM traffic per launch of the 320->320 3x3 conv at 64x64 (CFG batch 8): separate rocprofv3
# --pmc passes for FETCH_SIZE and WRITE_SIZE, fp16 halo (variant $2) and int8 halo (variant $3)
# usage: scripts/pmc_traffic.sh TAG [fp16 variant] [int8 variant]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/pmc_${1:-run}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for mode in f16 i8; do
  if [ $mode = f16 ]; then v=${2:-202}; flag=""; else v=${3:-142}; flag="--i8"; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${mode}_${ctr}_$v" -o run -- \
      python3 "$ROOT/scripts/roof_kernel.py" 10 $v $flag > "$OUT/${mode}_${ctr}_$v.log" 2>&1 || exit 99
  done
done
echo "[pmc] done"
