#!/bin/bash
# List every kernel with scratch (private memory) or VGPR spills in the libqdiff sources.
cd "$(dirname "$0")/../quantization---diffusion-models_amd/csrc" || exit 1
for f in *.hip; do
  extra=""
  [ "$f" = attn.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1"
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off $extra --cuda-device-only -c "$f" -o /tmp/_cs.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re
name = None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m: name = m.group(1); continue
    m = re.search(r"(ScratchSize \[bytes/lane\]|VGPRs Spill): (\d+)", l)
    if m and int(m.group(2)) > 0: print(sys.argv[1], name, m.group(1), m.group(2))
' "$f"
done
