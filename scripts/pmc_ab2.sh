#!/bin/bash
# A/B PMC passes (LDS / issue / memory-pipeline counters) of the dominant conv per GEMM variant
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcab2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-100 200}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/a_$v -o run -- python3 $ROOT/scripts/roof_kernel.py 5 $v > $OUT/a_$v.log 2>&1 || exit 99
  timeout -s KILL 90 rocprofv3 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $OUT/b_$v -o run -- python3 $ROOT/scripts/roof_kernel.py 5 $v > $OUT/b_$v.log 2>&1 || exit 99
done
echo done
