#!/bin/bash
# PMC passes (one counter group per run) of the attention kernel: bash scripts/pmc_attn.sh [d]
ROOT=$(pwd)
D=${1:-40}
OUT=$ROOT/gpurun_out/pmc_attn$D
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- python3 $ROOT/scripts/attn_one.py $D 5 > $OUT/a.log 2>&1 || exit 99
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $OUT/b -o run -- python3 $ROOT/scripts/attn_one.py $D 5 > $OUT/b.log 2>&1 || exit 98
echo done
