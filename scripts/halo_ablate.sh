#!/bin/bash
# Diagnostic libqdiff builds of the halo conv kernels with parts of their K loop removed
# (QD_HALO_ABL bits: 1 MFMAs, 2 weight DMA, 4 halo DMA, 8 barrier + vmcnt wait), linked with the
# in-tree objects, into scripts/ablate/libqdiff_abl<bits>.so (compiled in parallel).  Time them
# with scripts/halo_ablate.py on the GPU (QD_HALO_VAR selects the variant, default 200).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/quantization---diffusion-models_amd/csrc
mkdir -p "$ROOT/scripts/ablate"
for b in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -DQD_HALO_ABL=$b \
    -c "$C/gemm.hip" -o /tmp/gemm_abl$b.o &
done
wait
for b in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$C"/build/quant.o "$C"/build/norm.o /tmp/gemm_abl$b.o \
    "$C"/build/attn.o "$C"/build/mmdit.o "$C"/build/encdec.o -o "$ROOT/scripts/ablate/libqdiff_abl$b.so"
done
