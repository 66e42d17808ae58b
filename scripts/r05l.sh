#!/bin/bash
# round 5: PMC passes of the int8 short-K linears (K = N = 320 + residual; N = 2560 plain) and the
# int8-linear table re-tune with the persistent candidates
set -o pipefail
mkdir -p gpurun_out
PMC_TAG=_r05l_n320 timeout -k 10 400 bash scripts/pmc_shortk.sh > gpurun_out/r05l_pmc_n320.log 2>&1 || exit 11
PMC_TAG=_r05l_n2560 PMC_ARGS="--pmc-n 2560" timeout -k 10 400 bash scripts/pmc_shortk.sh > gpurun_out/r05l_pmc_n2560.log 2>&1 || exit 12
python3 scripts/pmc_reduce.py gpurun_out/pmc_shortk_r05l_n320 > gpurun_out/r05l_pmc_n320.txt 2>&1
python3 scripts/pmc_reduce.py gpurun_out/pmc_shortk_r05l_n2560 > gpurun_out/r05l_pmc_n2560.txt 2>&1
timeout -k 10 500 python3 -u scripts/tune_table.py --retune-i8-linear > gpurun_out/r05l_tune.log 2>&1 || exit 13
cp quantization---diffusion-models_amd/gemm_table.json gpurun_out/r05l_gemm_table.json
echo ok
