#!/bin/bash
# Issue / LDS / MFMA PMC passes (one counter group per run) of the SD1.5 64x64 320->320 conv for
# each halo variant: VARIANTS="140 202" bash scripts/pmc_halo.sh TAG   (reduce: scripts/pmc_reduce.py)
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_${1:-halo}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-140 202}; do
  QD_HALO_VAR=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/a_$v -o run -- python3 $ROOT/scripts/halo_ablate.py 0 > $OUT/a_$v.log 2>&1 || exit 99
  QD_HALO_VAR=$v timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $OUT/b_$v -o run -- python3 $ROOT/scripts/halo_ablate.py 0 > $OUT/b_$v.log 2>&1 || exit 98
  QD_HALO_VAR=$v timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM --output-format csv -d $OUT/c_$v -o run -- python3 $ROOT/scripts/halo_ablate.py 0 > $OUT/c_$v.log 2>&1 || exit 97
done
echo done
