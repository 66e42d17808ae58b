"""attn.to_out + residual -> LayerNorm at the SD1.5 64x64 level (M 32768, N = K = 320): the two
launches (tuned linear + layernorm / layernorm_i8) vs the row-complete LayerNorm epilogue
(kernels.linear_ln / linear_i8_ln) per tile variant, graph-replayed with the inputs rotated over 4
buffers.  usage: python scripts/ln_epi_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402


def graph_us(fns, iters=20):
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
    gen = torch.Generator().manual_seed(0)
    M, N, Kd, NB = 32768, 320, 320, 4
    xs = [torch.randn(M, Kd, generator=gen).half().to(dev) for _ in range(NB)]
    rs = [torch.randn(M, N, generator=gen).half().to(dev) for _ in range(NB)]
    w = (torch.randn(N, Kd, generator=gen) / Kd ** 0.5).half().to(dev)
    b = torch.randn(N, generator=gen).half().to(dev)
    gm = (1 + 0.1 * torch.randn(N, generator=gen)).half().to(dev)
    bt = (0.1 * torch.randn(N, generator=gen)).half().to(dev)
    qs = [K.quant_rows_i8(x) for x in xs]
    wq, sw16, _ = K.weight_quant(w, Kd, 8, want_dq=False)
    sw = sw16.float().view(-1).contiguous()
    for i8_out in (False, True):
        lnf = K.layernorm_i8 if i8_out else K.layernorm
        two = graph_us([lambda i=i: lnf(K.linear(xs[i], w, "f16", bias=b, residual=rs[i]), 1e-5, gm, bt)
                        for i in range(NB)])
        lin = graph_us([lambda i=i: K.linear(xs[i], w, "f16", bias=b, residual=rs[i]) for i in range(NB)])
        row = [f"fp16 two launches {two:.1f} us (linear {lin:.1f})"]
        for v in (None,) + K.LN_VARIANTS:
            K.force_gemm(v)
            try:
                t = graph_us([lambda i=i: K.linear_ln(xs[i], w, rs[i], gm, bt, 1e-5, bias=b, i8_out=i8_out)
                              for i in range(NB)])
            finally:
                K.force_gemm(None)
            row.append(f"fused[{v}] {t:.1f}")
        print(f"i8_out={i8_out}: " + " | ".join(row), flush=True)
        two8 = graph_us([lambda i=i: lnf(K.linear_i8(qs[i][0], qs[i][1], wq, sw, bias=b, residual=rs[i]), 1e-5, gm, bt)
                         for i in range(NB)])
        lin8 = graph_us([lambda i=i: K.linear_i8(qs[i][0], qs[i][1], wq, sw, bias=b, residual=rs[i]) for i in range(NB)])
        row = [f"int8 two launches {two8:.1f} us (linear {lin8:.1f})"]
        for v in (None,) + K.LN_I8_VARIANTS:
            K.force_gemm(v)
            try:
                t = graph_us([lambda i=i: K.linear_i8_ln(qs[i][0], qs[i][1], wq, sw, rs[i], gm, bt, 1e-5, bias=b,
                                                         i8_out=i8_out) for i in range(NB)])
            finally:
                K.force_gemm(None)
            row.append(f"fused[{v}] {t:.1f}")
        print(f"i8_out={i8_out}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
