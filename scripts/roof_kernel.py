"""Run ONLY the bench's dominant kernel (conv3x3 320->320 @64x64, CFG batch 8: M=32768, N=320,
K=2880) ITERS times, for rocprofv3 --pmc passes (HBM traffic per launch).
usage: python scripts/roof_kernel.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

if len(sys.argv) > 2:  # GEMM kernel family / tile override (qd_gemm_force id), for A/B profiles
    K.force_gemm(int(sys.argv[2]))

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
n, h, w, c = 8, 64, 64, 320
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(n, h, w, c, generator=g).half().to(dev)
wt = (torch.randn(c, 3, 3, c, generator=g) / 54).half().to(dev)
b = torch.zeros(c, dtype=torch.float16, device=dev)
amax = torch.empty(n * c, dtype=torch.float32, device=dev)
for _ in range(iters):
    K.conv2d_nhwc(x, wt, c, 1, 1, bias=b, amax=amax)
torch.cuda.synchronize()
print("algorithmic bytes per launch:", x.numel() * 2 + wt.numel() * 2 + n * h * w * c * 2)
