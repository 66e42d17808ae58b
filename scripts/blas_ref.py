"""Reference point only (not the product path): torch.matmul (hipBLASLt / rocBLAS) rate on the
path's dominant GEMM shapes, next to libqdiff's kernel for the same shape."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import kernels as K

def t(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); [fn() for _ in range(iters)]; e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / iters

dev = "cuda:0"
for (m, n, k) in ((8192, 9728, 2432), (8192, 2432, 9728), (4096, 7296, 2432), (32768, 320, 2880), (8192, 1280, 1280), (32768, 2560, 320)):
    a = torch.randn(m, k, device=dev).half()
    w = (torch.randn(n, k, device=dev) / k ** 0.5).half()
    ms_b = t(lambda: torch.matmul(a, w.t()))
    ms_q = t(lambda: K.linear(a, w, "f16"))
    f = 2 * m * n * k
    print(f"M={m} N={n} K={k}: torch.matmul {ms_b*1e3:.1f} us {f/ms_b/1e9:.0f} TFLOP/s | libqdiff {ms_q*1e3:.1f} us {f/ms_q/1e9:.0f} TFLOP/s", flush=True)

# per-variant sweep (qd_gemm_force ids) on the same shapes
print("variant sweep (TFLOP/s):")
for (m, n, k) in ((8192, 9728, 2432), (8192, 2432, 9728), (4096, 7296, 2432), (32768, 320, 2880), (8192, 1280, 1280), (32768, 2560, 320), (32768, 960, 320), (2048, 1280, 11520)):
    a = torch.randn(m, k, device=dev).half()
    w = (torch.randn(n, k, device=dev) / k ** 0.5).half()
    f = 2 * m * n * k
    row = []
    for v in (100, 101, 103, 106, 109, 300, 301, 302, 303, 304):
        K.force_gemm(v)
        try:
            ms = t(lambda: K.linear(a, w, "f16"))
            row.append(f"{v}:{f / ms / 1e9:.0f}")
        except RuntimeError as e:
            row.append(f"{v}:err")
        K.force_gemm(None)
    print(f"M={m} N={n} K={k}: " + " ".join(row), flush=True)
