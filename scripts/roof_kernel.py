"""Run ONLY the bench's dominant kernel (conv3x3 320->320 @64x64, CFG batch 8: M=32768, N=320,
K=2880) ITERS times, in the form the captured step launches it (bench.dominant_kernel_roofline), for
rocprofv3 --pmc passes (HBM traffic per launch).
usage: python scripts/roof_kernel.py [iters] [variant] [--i8]
  fp16: bias + the output fake-quant's amax epilogue into a pre-zeroed buffer (no zero-fill launch)
  --i8: the int8-MFMA mode's resnet conv1 (int8 codes, one scale per sample, per-channel weight codes)
        with bias + the time-embedding add + the consumer GroupNorm's slot statistics"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
i8 = "--i8" in sys.argv
if len(args) > 1:  # GEMM kernel family / tile override (qd_gemm_force id), for A/B profiles
    K.force_gemm(int(args[1]))

iters = int(args[0]) if args else 10
dev = torch.device("cuda:0")
n, h, w, c = 8, 64, 64, 320
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(n, h, w, c, generator=g).half().to(dev)
wt = (torch.randn(c, 3, 3, c, generator=g) / 54).half().to(dev)
b = torch.zeros(c, dtype=torch.float16, device=dev)
amax = torch.zeros(n * c, dtype=torch.float32, device=dev)
if i8:
    xq, sa = K.quant_samples_i8(x)
    wq = torch.randint(-127, 128, (c, 3, 3, c), generator=g, dtype=torch.int8).to(dev)
    sw = torch.full((c,), 1e-3, dtype=torch.float32, device=dev)
    temb = (torch.randn(n, c, generator=g) * 0.1).half().to(dev)
    for _ in range(iters):
        K.conv2d_i8(xq, sa, wq, sw, c, 1, 1, bias=b, chan_add=temb, gn_stats=True)
    torch.cuda.synchronize()
    # codes + weights + fp16 output + the slot moments (one float4 per 64-row slot and column)
    print("algorithmic bytes per launch:", xq.numel() + wq.numel() + n * h * w * c * 2 + n * h * w // 64 * c * 16)
else:
    for _ in range(iters):
        K.conv2d_nhwc(x, wt, c, 1, 1, bias=b, amax=amax, amax_zeroed=True)
    torch.cuda.synchronize()
    print("algorithmic bytes per launch:", x.numel() * 2 + wt.numel() * 2 + n * h * w * c * 2)
