#!/bin/bash
# round 5: the post-residual amax at the split-K levels (k_splitk_reduce takes it after the residual
# add): its kernel tests, the UNet tests, then the new (16x16 / 8x8 level) keys added to the table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -rf \
  tests/ -m gpu -k "post_residual or groupnorm or gn_" > gpurun_out/r05z_post_tests.log 2>&1 || exit 11
tail -2 gpurun_out/r05z_post_tests.log
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 --timeout-method thread -rf tests/test_gpu_unet.py \
  > gpurun_out/r05z_unet_tests.log 2>&1 || exit 12
tail -2 gpurun_out/r05z_unet_tests.log
timeout -k 10 420 python3 -u scripts/tune_table.py --add --models sd15,sdxl > gpurun_out/r05z_tune.log 2>&1 || exit 13
cp quantization---diffusion-models_amd/gemm_table.json gpurun_out/r05z_gemm_table.json
tail -3 gpurun_out/r05z_tune.log
