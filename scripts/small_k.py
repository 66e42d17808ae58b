"""Level-0 (M = 32768, K = 320) GEMM shapes of the SD1.5 UNet at CFG batch 8: per-variant time
with and without the fused GEGLU epilogue, next to torch.matmul (reference point only)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import kernels as K


def t(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); [fn() for _ in range(iters)]; e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


dev = "cuda:0"
for (m, n, k, geglu) in ((32768, 2560, 320, True), (32768, 2560, 320, False), (32768, 960, 320, False),
                         (32768, 320, 320, False), (32768, 320, 1280, False), (8192, 5120, 640, True)):
    a = torch.randn(m, k, device=dev).half()
    w = (torch.randn(n, k, device=dev) / k ** 0.5).half()
    b = torch.randn(n, device=dev).half()
    ref = t(lambda: torch.matmul(a, w.t()))
    row = []
    for v in list(K.REG_VARIANTS) + list(K.DMA_VARIANTS):
        K.force_gemm(v)
        try:
            us = t(lambda: K.linear(a, w, "f16", bias=b, geglu=geglu))
            row.append(f"{v}:{us:.1f}")
        except RuntimeError:
            row.append(f"{v}:err")
        K.force_gemm(None)
    print(f"M={m} N={n} K={k} geglu={geglu}: matmul {ref:.1f}us | " + " ".join(row), flush=True)
