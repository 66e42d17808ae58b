"""Cost of the AMAX epilogue (per-(sample, column) atomic max) on the UNet's conv shapes:
the same conv with and without it, per forced GEMM variant (time under rocprofv3 --kernel-trace
or with the events printed here)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import kernels as K

dev = "cuda:0"
for (n, h, w, c) in ((8, 64, 64, 320), (8, 32, 32, 640), (8, 16, 16, 1280)):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(n, h, w, c, generator=g).half().to(dev)
    wt = (torch.randn(c, 3, 3, c, generator=g) / (3 * c ** 0.5)).half().to(dev)
    b = torch.zeros(c, dtype=torch.float16, device=dev)
    am = torch.zeros(n * c, dtype=torch.float32, device=dev)
    row = []
    for v in (106, 200, 300):
        for use_am in (False, True):
            K.force_gemm(v)
            try:
                fn = lambda: K.conv2d_nhwc(x, wt, c, 1, 1, bias=b, amax=am if use_am else None, amax_zeroed=use_am)
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record(); e1.synchronize()
                row.append(f"{v}{'+am' if use_am else ''}:{e0.elapsed_time(e1) / 20 * 1e3:.1f}")
            except RuntimeError:
                row.append(f"{v}:err")
            finally:
                K.force_gemm(None)
    print((n, h, w, c), " ".join(row), flush=True)
