"""Epilogue ablation of the int8 linears on the SD1.5 64x64-level shapes (ff.net.2: M 32768, K 1280,
N 320 with bias + residual + post-residual amax; the K = N = 320 projections): per variant, the GPU
time of the plain GEMM, + bias, + residual, + the post-residual per-(sample, column) amax, warm (graph
replay of back-to-back launches) and cold (a 512 MB flush before each launch, HIP events around the
launch alone), beside a device copy of the same byte volume.

usage: python scripts/epi_ablate.py [--variants 110 113 ...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def warm_time(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e3)
    return best


FLUSH = None


def cold_time(fn, reps=5):
    global FLUSH
    if FLUSH is None:
        FLUSH = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    fn()
    ts = []
    for _ in range(reps):
        FLUSH.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="*", type=int, default=[])
    a = ap.parse_args()
    variants = a.variants or list(K.I8_VARIANTS)
    g = torch.Generator(device="cpu").manual_seed(0)
    for (m, n, k, rps) in [(32768, 320, 1280, 4096), (32768, 320, 320, 4096)]:
        x = torch.randn(m, k, generator=g).half().to(dev)
        wt = (torch.randn(n, k, generator=g) / k ** 0.5).half().to(dev)
        b = (0.1 * torch.randn(n, generator=g)).half().to(dev)
        res = torch.randn(m, n, generator=g).half().to(dev)
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(wt, k, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()
        am = torch.zeros(m // rps * n, dtype=torch.float32, device=dev)
        forms = {
            "plain": lambda: K.linear_i8(xq, sa, wq, sw),
            "bias": lambda: K.linear_i8(xq, sa, wq, sw, bias=b),
            "bias+res": lambda: K.linear_i8(xq, sa, wq, sw, bias=b, residual=res),
            "bias+res+amax": lambda: K.linear_i8(xq, sa, wq, sw, bias=b, residual=res, amax=am,
                                                 rows_per_sample=rps, amax_post=True),
        }
        mb_in, mb_out = m * k / 1e6, m * n * 2 / 1e6
        src = torch.empty(int((mb_in + 2 * mb_out) * 1e6) // 2, dtype=torch.float16, device=dev)
        dst = torch.empty_like(src)
        cp = lambda: dst.copy_(src)
        print(f"M {m} N {n} K {k}: A {mb_in:.1f} MB, out {mb_out:.1f} MB (+ residual {mb_out:.1f} MB); "
              f"copy of {src.numel() * 2 / 1e6:.1f} MB: warm {warm_time(cp):.1f} us, cold {cold_time(cp):.1f} us",
              flush=True)
        for name, fn in forms.items():
            cells = []
            for v in variants:
                K.force_gemm(v)
                try:
                    cells.append(f"{v}:{warm_time(fn):.1f}/{cold_time(fn):.1f}")
                except RuntimeError:
                    cells.append(f"{v}:err")
                finally:
                    K.force_gemm(None)
            print(f"  {name:14s} warm/cold us  " + " ".join(cells), flush=True)


if __name__ == "__main__":
    main()
