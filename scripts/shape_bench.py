"""Per-variant GPU time of the SD1.5 CFG-batch-8 GEMM / conv shapes, launch overhead excluded:
each (shape, variant) is captured as a HIP graph of `iters` back-to-back calls and replayed.
usage: python scripts/shape_bench.py [--int8] [--iters 20] [--only conv|linear] [--amax] [--w4 [--mscale 2]]
(--amax: the fp16 convs with the per-(sample, channel) output-amax epilogue of the W8A8 path;
 --w4: the linears as W4A16 group-128 codes - packed int4 through the register tile and the LDS-DMA /
 ping-pong int4 stages vs the fp16 dequantized buffer through every fp16 family; --mscale 2 = C3's
 CFG batch 16)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

# (n, h, w, cin, cout, k, stride, count per eval)
CONVS = [(8, 64, 64, 320, 320, 3, 1, 7), (8, 32, 32, 640, 640, 3, 1, 6), (8, 16, 16, 1280, 1280, 3, 1, 7),
         (8, 8, 8, 1280, 1280, 3, 1, 8), (8, 64, 64, 640, 320, 3, 1, 2), (8, 64, 64, 960, 320, 3, 1, 1),
         (8, 32, 32, 1280, 640, 3, 1, 2), (8, 16, 16, 2560, 1280, 3, 1, 2), (8, 32, 32, 320, 640, 3, 1, 1)]
# the down-block samplers (stride 2): --stride2 runs only these
CONVS_S2 = [(8, 64, 64, 320, 320, 3, 2, 1), (8, 32, 32, 640, 640, 3, 2, 1), (8, 16, 16, 1280, 1280, 3, 2, 1)]
# (M, N, K, geglu, count per eval)
LINS = [(32768, 320, 320, False, 25), (32768, 960, 320, False, 5), (32768, 2560, 320, True, 5),
        (32768, 320, 1280, False, 5), (8192, 640, 640, False, 25), (8192, 5120, 640, True, 5),
        (8192, 640, 2560, False, 5), (2048, 1280, 1280, False, 25), (2048, 10240, 1280, True, 6),
        (2048, 1280, 5120, False, 6)]


def graph_time(fn, iters):
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


def run_variants(fn, variants, iters):
    out = {}
    for v in variants:
        K.force_gemm(v)
        try:
            out[v] = graph_time(fn, iters)
        except RuntimeError:
            out[v] = None
        finally:
            K.force_gemm(None)
    return out


def fmt(res, flops):
    best = min((t for t in res.values() if t), default=None)
    cells = []
    for v, t in res.items():
        cells.append(f"{v}:{'err' if t is None else f'{t:.1f}'}{'*' if t == best else ''}")
    return f"best {best:.1f} us ({flops / best / 1e6:.0f} T/s) | " + " ".join(cells)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--int8", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None, choices=["conv", "linear"])
    ap.add_argument("--amax", action="store_true")
    ap.add_argument("--w4", action="store_true")
    ap.add_argument("--mscale", type=int, default=1)
    ap.add_argument("--stride2", action="store_true")
    a = ap.parse_args()
    if a.w4:
        return w4_linears(a)
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    if a.int8:
        variants = list(K.I8_VARIANTS)
    else:
        variants = list(K.REG_VARIANTS) + list(K.DMA_VARIANTS)
    if a.only != "linear":
        for (n, h, w, ci, co, k, s, cnt) in (CONVS_S2 if a.stride2 else CONVS):
            x = torch.randn(n, h, w, ci, generator=g).half().to(dev)
            wt = (torch.randn(co, k, k, ci, generator=g) / (k * k * ci) ** 0.5).half().to(dev)
            b = torch.zeros(co, dtype=torch.float16, device=dev)
            flops = 2.0 * n * h * w * co * k * k * ci / (s * s)
            if a.int8:
                xq, sa = K.quant_samples_i8(x)
                wq, sw16, _ = K.weight_quant(wt.view(co, -1).contiguous(), k * k * ci, 8, want_dq=False)
                wq = wq.view(co, k, k, ci)
                sw = sw16.float().view(-1).contiguous()
                res = run_variants(lambda: K.conv2d_i8(xq, sa, wq, sw, ci, s, k // 2, bias=b), variants, a.iters)
            else:
                vs = variants + (list(K.HALO_VARIANTS) if k == 3 and s == 1 else [])
                am = torch.zeros(n * co, dtype=torch.float32, device=dev) if a.amax else None
                res = run_variants(lambda: K.conv2d_nhwc(x, wt, ci, s, k // 2, bias=b, amax=am), vs, a.iters)
            print(f"conv ({n},{h},{w},{ci},{co},{k}){' amax' if a.amax else ''} x{cnt}: " + fmt(res, flops), flush=True)
    if a.only != "conv" and not a.stride2:
        for (m, nn, kk, geglu, cnt) in LINS:
            x = torch.randn(m, kk, generator=g).half().to(dev)
            wt = (torch.randn(nn, kk, generator=g) / kk ** 0.5).half().to(dev)
            b = torch.zeros(nn, dtype=torch.float16, device=dev)
            flops = 2.0 * m * nn * kk
            if a.int8:
                xq, sa = K.quant_rows_i8(x)
                wq, sw16, _ = K.weight_quant(wt, kk, 8, want_dq=False)
                sw = sw16.float().view(-1).contiguous()
                res = run_variants(lambda: K.linear_i8(xq, sa, wq, sw, bias=b, geglu=geglu), variants, a.iters)
            else:
                res = run_variants(lambda: K.linear(x, wt, bias=b, geglu=geglu), variants, a.iters)
            print(f"linear ({m},{nn},{kk}{',geglu' if geglu else ''}) x{cnt}: " + fmt(res, flops), flush=True)


def w4_linears(a):
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    f16v = list(K.REG_VARIANTS) + list(K.DMA_VARIANTS)
    i4v = list(K.REG_VARIANTS) + list(K.W4_VARIANTS)
    tot16 = tot4 = 0.0
    for (m, nn, kk, geglu, cnt) in LINS:
        m *= a.mscale
        x = torch.randn(m, kk, generator=g).half().to(dev)
        wt = (torch.randn(nn, kk, generator=g) / kk ** 0.5).half().to(dev)
        b = torch.zeros(nn, dtype=torch.float16, device=dev)
        gs = 128
        while kk % gs:
            gs -= 32
        codes, sc, wdq = K.weight_quant(wt, gs, 4)
        packed = K.pack_int4(codes)
        flops = 2.0 * m * nn * kk
        r16 = run_variants(lambda: K.linear(x, wdq, "f16", bias=b, geglu=geglu), f16v, a.iters)
        r4 = run_variants(lambda: K.linear(x, packed, "i4", sc, gs, bias=b, geglu=geglu), i4v, a.iters)
        b16 = min(t for t in r16.values() if t)
        b4 = min(t for t in r4.values() if t)
        tot16 += cnt * b16
        tot4 += cnt * b4
        print(f"linear ({m},{nn},{kk}{',geglu' if geglu else ''}) x{cnt} g{gs}: fp16 buffer {fmt(r16, flops)}", flush=True)
        print(f"    int4 codes {fmt(r4, flops)}  -> i4/f16 {b4 / b16:.3f}", flush=True)
    print(f"sum over one eval's linears: fp16 buffer {tot16:.0f} us, int4 codes {tot4:.0f} us", flush=True)


if __name__ == "__main__":
    main()
