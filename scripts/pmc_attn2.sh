#!/bin/bash
# PMC passes of the d = 40 attention: 16x16x32 kernel (qd_attn_force 6) vs the 32x32x16 one (default)
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for cfg in 6 0; do
  OUT=$ROOT/gpurun_out/pmc_attn_cfg$cfg
  mkdir -p $OUT
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- python3 $ROOT/scripts/attn_one.py 40 5 $cfg > $OUT/a.log 2>&1 || exit 99
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $OUT/b -o run -- python3 $ROOT/scripts/attn_one.py 40 5 $cfg > $OUT/b.log 2>&1 || exit 98
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_EXP --output-format csv -d $OUT/c -o run -- python3 $ROOT/scripts/attn_one.py 40 5 $cfg > $OUT/c.log 2>&1 || exit 97
done
echo done
