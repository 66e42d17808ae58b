"""Diagnostic: time GEMM variants on the dominant conv and a large linear with a given libqdiff
build (e.g. scripts/ablate/libqdiff.so built with -DQD_ABLATE_NO_MFMA: staging + fragment reads
only) to separate load-pipeline time from MFMA time.
usage: python scripts/ablate_gemm.py [path/to/libqdiff.so]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
from qdiff import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


x = torch.randn(8, 64, 64, 320, device=dev).half()
wt = (torch.randn(320, 3, 3, 320, device=dev) * 0.02).half()
b = torch.zeros(320, device=dev).half()
am = torch.empty(8 * 320, device=dev)
xl = torch.randn(8192, 640, device=dev).half()
wl = (torch.randn(5120, 640, device=dev) * 0.02).half()
print("lib:", _lib.LIB_PATH)
for v in (0, 100, 101, 103, 106, 109):
    K.force_gemm(v)
    tc = timeit(lambda: K.conv2d_nhwc(x, wt, 320, 1, 1, bias=b, amax=am))
    tl = timeit(lambda: K.linear(xl, wl))
    print(f"variant {v:3d}: conv3x3 64^2 320 {tc:7.1f} us ({60.4e3 / tc:6.0f} TF)   linear 8192x640x5120 {tl:7.1f} us "
          f"({2 * 8192 * 640 * 5120 / tl / 1e6:6.0f} TF)", flush=True)
