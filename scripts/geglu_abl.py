"""Ablation timing of the short-K GEMMs (SD1.5 64x64 level): run once with the normal library and
once with QD_LIB_PATH pointing at a diagnostic build (e.g. -DQD_ABLATE_EPI_STORES: the direct
epilogue computes everything but drops its stores) - the difference is what the output stores cost.
usage: [QD_LIB_PATH=...] python scripts/geglu_abl.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402


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


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    M, Kd, N = 32768, 320, 2560
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(dev)
    b = torch.randn(N, generator=g).half().to(dev)
    xq, sa = K.quant_rows_i8(x)
    wq, sw16, _ = K.weight_quant(w, Kd, 8, want_dq=False)
    sw = sw16.float().view(-1).contiguous()
    cases = [("f16 geglu", lambda: K.linear(x, w, "f16", bias=b, geglu=True)),
             ("f16 plain", lambda: K.linear(x, w, "f16", bias=b)),
             ("i8 geglu", lambda: K.linear_i8(xq, sa, wq, sw, bias=b, geglu=True)),
             ("i8 plain", lambda: K.linear_i8(xq, sa, wq, sw, bias=b))]
    lib = os.environ.get("QD_LIB_PATH", "default")
    for name, fn in cases:
        fn()
        ts = [timeit(fn) for _ in range(3)]
        print(f"[{os.path.basename(lib)}] {name:10s} {statistics.median(ts):7.1f} us", flush=True)
    print("choices:", K.gemm_choices(used_only=True))


if __name__ == "__main__":
    main()
