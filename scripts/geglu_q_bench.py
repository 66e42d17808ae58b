"""int8 GEGLU at the SD1.5 64x64 level (M 32768, K 320, N 2560): the two-launch path
(linear_i8(geglu=True) + quant_rows_i8) against the fused qd_linear_i8_geglu_q (both wave layouts),
HIP-event timed, interleaved rounds in one process.  usage: python scripts/geglu_q_bench.py"""
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

    def two():
        return K.quant_rows_i8(K.linear_i8(xq, sa, wq, sw, bias=b, geglu=True))

    def gemm_only():
        return K.linear_i8(xq, sa, wq, sw, bias=b, geglu=True)

    def fused(v):
        K.force_gemm(v)
        try:
            return K.linear_i8_geglu_q(xq, sa, wq, sw, bias=b)
        finally:
            K.force_gemm(None)
    a = two()
    for v in (150, 151):
        c = fused(v)
        print(f"variant {v} bit-identical:", torch.equal(a[0], c[0]) and torch.equal(a[1], c[1]), flush=True)
    res = {k: [] for k in ("two launches", "GEGLU GEMM alone", "fused 150 (64 rows, 8 waves)",
                           "fused 151 (64 rows, 4 waves)")}
    for _ in range(4):
        res["two launches"].append(timeit(two))
        res["GEGLU GEMM alone"].append(timeit(gemm_only))
        res["fused 150 (64 rows, 8 waves)"].append(timeit(lambda: fused(150)))
        res["fused 151 (64 rows, 4 waves)"].append(timeit(lambda: fused(151)))
    for k, v in res.items():
        print(f"{k:24s} median {statistics.median(v):7.1f} us  (min {min(v):.1f})", flush=True)


if __name__ == "__main__":
    main()
