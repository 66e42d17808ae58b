#!/bin/bash
# round 5: static issue priority for the younger half of k_attn32's 8-wave block - same-box A/B of
# the attention shapes (A = the library without it, B = the tree's), alternating 3 rounds
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  QD_LIB_PATH=$PWD/scripts/ab/libqdiff_r05zh.so timeout -k 10 120 python3 scripts/attn_bench.py > gpurun_out/r05zi_A$r.log 2>&1 || exit 11
  timeout -k 10 120 python3 scripts/attn_bench.py > gpurun_out/r05zi_B$r.log 2>&1 || exit 12
done
grep -h "sq=4096 skv=4096 h=8 d=40\|sq=4096 skv=77" gpurun_out/r05zi_A*.log gpurun_out/r05zi_B*.log
