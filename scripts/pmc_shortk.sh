#!/bin/bash
# PMC passes of the tuned int8 short-K linear (M 32768, N 320, K 320, + residual): stall / issue
# counters and HBM traffic, one counter group per rocprofv3 run
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_shortk${PMC_TAG:-}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$1 -o run -- python3 $ROOT/scripts/shortk_i8.py --pmc $PMC_ARGS > $OUT/$1.log 2>&1; }
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit 99
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAVES || exit 98
run FETCH_SIZE || exit 97
run WRITE_SIZE || exit 96
run TCC_HIT_sum TCC_MISS_sum || exit 95
echo done
