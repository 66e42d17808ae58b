"""Feed-forward output GEMMs (ff.net.2: K = 4C, N = C, + residual) of the SD1.5 levels at the CFG
batch 8: tuned time and every forced fp16 variant, hot (one A) and graph-replayed with A rotated
over distinct buffers (the UNet's A is the GEGLU output just written, never re-read).
usage: python scripts/ffout_sweep.py"""
import os
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


def graph_us(fns, iters=10):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fns:
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters / len(fns) * 1e3


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    NA = 4
    for (m, n, k) in ((32768, 320, 1280), (8192, 640, 2560), (2048, 1280, 5120)):
        xs = [torch.randn(m, k, generator=g).half().to(dev) for _ in range(NA)]
        w = (torch.randn(n, k, generator=g) / k ** 0.5).half().to(dev)
        b = torch.randn(n, generator=g).half().to(dev)
        r = torch.randn(m, n, generator=g).half().to(dev)
        outs = [torch.empty(m, n, dtype=torch.float16, device=dev) for _ in range(NA)]
        hot = timeit(lambda: K.linear(xs[0], w, "f16", bias=b, residual=r, out=outs[0]))
        cold = graph_us([lambda i=i: K.linear(xs[i], w, "f16", bias=b, residual=r, out=outs[i]) for i in range(NA)])
        bl = graph_us([lambda i=i: torch.addmm(r, xs[i], w.t(), out=outs[i]) for i in range(NA)])
        bl_hot = timeit(lambda: torch.addmm(r, xs[0], w.t(), out=outs[0]))
        print(f"    torch.addmm (hipBLASLt, + residual): hot {bl_hot:.1f} us, graph cold {bl:.1f} us", flush=True)
        mb = (m * k + 2 * m * n) * 2 / 1e6
        print(f"M {m} N {n} K {k} (+res, {mb:.0f} MB, {2 * m * n * k / 1e9:.1f} GFLOP): tuned hot {hot:.1f} us, "
              f"graph cold {cold:.1f} us", flush=True)
        row = []
        for v in K.REG_VARIANTS + K.DMA_VARIANTS + (110, 111, 112, 113):
            K.force_gemm(v)
            try:
                t = graph_us([lambda i=i: K.linear(xs[i], w, "f16", bias=b, residual=r, out=outs[i])
                              for i in range(NA)])
                row.append(f"{v}:{t:.1f}")
            except Exception:  # noqa: BLE001
                row.append(f"{v}:x")
            K.force_gemm(None)
        print("    forced (graph, cold A): " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
