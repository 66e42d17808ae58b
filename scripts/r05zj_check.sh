#!/bin/bash
# round 5: attention tests on the static-priority build, then the final measurements
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 --timeout-method thread -rf tests -m gpu \
  -k "attention or c2 or pixel or golden" > gpurun_out/r05zj_tests.log 2>&1 || exit 11
tail -2 gpurun_out/r05zj_tests.log
bash scripts/r05_final.sh r05zj || exit 12
