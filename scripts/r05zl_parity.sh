#!/bin/bash
# round 5: the parity / determinism / UNet files on the re-tuned table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread -rf tests/test_gpu_pixel.py \
  tests/test_gpu_c2.py tests/test_gpu_golden_modules.py tests/test_gpu_configs.py tests/test_gpu_unet.py \
  tests/test_gpu_determinism.py tests/test_gpu_int8_accuracy.py tests/test_gpu_dist.py tests/test_gpu_sdxl.py \
  > gpurun_out/r05zl_tests.log 2>&1 || exit 11
tail -3 gpurun_out/r05zl_tests.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05zl_smoke.log 2>&1 || exit 12
tail -1 gpurun_out/r05zl_smoke.log
