#!/bin/bash
# A/B PMC passes of the dominant conv for several GEMM variants
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for v in -1 100 109; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq_$v -o run -- python3 $ROOT/scripts/roof_kernel.py 5 $v > $OUT/sq_$v.log 2>&1 || exit 99
  timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tc_$v -o run -- python3 $ROOT/scripts/roof_kernel.py 5 $v > $OUT/tc_$v.log 2>&1 || echo "tc pass failed $v"
done
echo done
