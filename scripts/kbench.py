"""Per-kernel microbenchmarks on the SD1.5 UNet shapes (CFG batch 8, 512x512) - HIP-event timed.

usage: python scripts/kbench.py [attn] [gn] [conv] [linear]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream()
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).half()


def bench_attn():
    b, heads = 8, 8
    for sq, skv, d in [(4096, 4096, 40), (4096, 77, 40), (1024, 1024, 80), (1024, 77, 80), (256, 256, 160),
                       (256, 77, 160), (64, 64, 160), (64, 77, 160)]:
        c = heads * d
        q, k, v = rnd(b, sq, c), rnd(b, skv, c), rnd(b, skv, c)
        us = timeit(lambda: K.attention(q, k, v, heads))
        fl = 4.0 * b * heads * sq * skv * d
        print(f"attn sq={sq:5d} skv={skv:5d} d={d:3d}: {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s", flush=True)


def bench_gn():
    for n, hw, c, silu, q in [(8, 4096, 320, True, 8), (8, 4096, 960, True, 8), (8, 1024, 640, True, 8),
                              (8, 256, 1280, True, 8), (8, 64, 1280, True, 8), (8, 4096, 320, False, 0)]:
        x = rnd(n, hw, c)
        gam, bet = rnd(c), rnd(c)
        us = timeit(lambda: K.groupnorm_nhwc(x, 32, 1e-5, gam, bet, silu=silu, q_bits=q))
        by = 2.0 * n * hw * c * 2
        print(f"gn n={n} hw={hw:5d} c={c:5d} q={q}: {us:8.1f} us  {by / us / 1e3:7.1f} GB/s (2 passes)", flush=True)


def bench_conv():
    for n, h, ci, co, k in [(8, 64, 320, 320, 3), (8, 32, 640, 640, 3), (8, 16, 1280, 1280, 3),
                            (8, 8, 1280, 1280, 3), (8, 64, 640, 320, 3), (8, 32, 1920, 640, 3),
                            (8, 16, 2560, 1280, 3), (8, 64, 320, 320, 1)]:
        x = rnd(n, h, h, ci)
        wt = rnd(co, k, k, ci, scale=0.02)
        bias = rnd(co)
        amax = torch.empty(n * co, dtype=torch.float32, device=dev)
        us = timeit(lambda: K.conv2d_nhwc(x, wt, ci, 1, k // 2, bias=bias, amax=amax))
        fl = 2.0 * n * h * h * co * ci * k * k
        print(f"conv n={n} {h}x{h} {ci:4d}->{co:4d} k{k}: {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s", flush=True)


def bench_linear():
    for m, kk, nn in [(32768, 320, 320), (32768, 320, 2560), (32768, 1280, 320), (8192, 640, 640),
                      (8192, 640, 5120), (8192, 2560, 640), (2048, 1280, 1280), (2048, 1280, 10240),
                      (2048, 5120, 1280), (616, 768, 320)]:
        x = rnd(m, kk)
        w = rnd(nn, kk, scale=0.02)
        us = timeit(lambda: K.linear(x, w))
        fl = 2.0 * m * kk * nn
        print(f"linear M={m:6d} K={kk:5d} N={nn:6d}: {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s", flush=True)




def bench_sweep():
    """Every GEMM kernel family / tile (qd_gemm_force) on the SD1.5 conv and linear shapes."""
    from qdiff import _lib
    variants = [-1, 100, 101, 106, 109, 200, 201]
    convs = [(8, 64, 320, 320, 3), (8, 32, 640, 640, 3), (8, 16, 1280, 1280, 3), (8, 8, 1280, 1280, 3),
             (8, 64, 640, 320, 3), (8, 32, 1920, 640, 3), (8, 16, 2560, 1280, 3), (8, 64, 320, 320, 1)]
    for n, h, ci, co, k in convs:
        x = rnd(n, h, h, ci)
        wt = rnd(co, k, k, ci, scale=0.02)
        bias = rnd(co)
        amax = torch.empty(n * co, dtype=torch.float32, device=dev)
        fl = 2.0 * n * h * h * co * ci * k * k
        row = []
        for v in variants:
            K.force_gemm(v)
            us = timeit(lambda: K.conv2d_nhwc(x, wt, ci, 1, k // 2, bias=bias, amax=amax))
            row.append(f"{v}:{fl / us / 1e6:6.0f}")
        print(f"conv {h}x{h} {ci}->{co} k{k}: " + " ".join(row), flush=True)
    for m, kk, nn in [(32768, 320, 320), (32768, 320, 2560), (32768, 1280, 320), (8192, 640, 640),
                      (8192, 640, 5120), (8192, 2560, 640), (2048, 1280, 1280), (2048, 1280, 10240),
                      (2048, 5120, 1280)]:
        x = rnd(m, kk)
        w = rnd(nn, kk, scale=0.02)
        fl = 2.0 * m * kk * nn
        row = []
        for v in variants:
            K.force_gemm(v)
            us = timeit(lambda: K.linear(x, w))
            row.append(f"{v}:{fl / us / 1e6:6.0f}")
        print(f"linear {m}x{kk}x{nn}: " + " ".join(row), flush=True)
    K.force_gemm(None)


if __name__ == "__main__":
    which = sys.argv[1:] or ["attn", "gn", "conv", "linear"]
    for w in which:
        globals()[f"bench_{w}"]()
