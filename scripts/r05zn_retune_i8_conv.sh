#!/bin/bash
# round 5: re-tune the int8 convs with this round's kernels, then a
# same-box A/B of the committed table ("prev") against the re-tuned one ("new"), 3 rounds
set -o pipefail
mkdir -p gpurun_out scripts/ab
cp quantization---diffusion-models_amd/gemm_table.json scripts/ab/gemm_table_r05zn_prev.json
timeout -k 10 400 python3 -u scripts/tune_table.py --retune-i8-conv > gpurun_out/r05zn_tune.log 2>&1 || exit 11
cp quantization---diffusion-models_amd/gemm_table.json gpurun_out/r05zn_gemm_table.json
tail -2 gpurun_out/r05zn_tune.log
timeout -k 10 900 bash scripts/ab_env.sh QD_GEMM_TABLE=$PWD/scripts/ab/gemm_table_r05zn_prev.json 3 > gpurun_out/r05zn_ab.log 2>&1 || exit 12
cat gpurun_out/r05zn_ab.log
