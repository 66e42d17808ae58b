"""fp16 3x3 conv at the SD1.5 levels (CFG batch 8) in the forms the fake-quant UNet runs them: plain,
+ per-(sample, channel) output amax (the reference's output fake-quant needs it), + residual,
graph-replayed (weights rotated over distinct copies so they are not L2/MALL-resident), each
tuned; shows what the amax / residual epilogues and cold weights cost per level.
usage: python scripts/conv_epi_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402


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
    gen = torch.Generator(device="cpu").manual_seed(0)
    NW = 8  # distinct weight copies per shape (a UNet eval never reuses a conv's weights)
    for (n, h, ci, co) in ((8, 64, 320, 320), (8, 32, 640, 640), (8, 16, 1280, 1280), (8, 8, 1280, 1280)):
        x = torch.randn(n, h, h, ci, generator=gen).half().to(dev)
        ws = [(torch.randn(co, 3, 3, ci, generator=gen) / (9 * ci) ** 0.5).half().to(dev) for _ in range(NW)]
        b = torch.zeros(co, dtype=torch.float16, device=dev)
        r = torch.randn(n, h, h, co, generator=gen).half().to(dev)
        outs = [torch.empty(n, h, h, co, dtype=torch.float16, device=dev) for _ in range(NW)]
        am = [torch.zeros(n * co, dtype=torch.float32, device=dev) for _ in range(NW)]
        rows = []
        for label, kw in (("plain", {}), ("amax", {"amax": True}), ("res", {"residual": r}),
                          ("amax+res", {"amax": True, "residual": r})):
            def mk(i, kw=kw):
                a = am[i] if kw.get("amax") else None
                return lambda: K.conv2d_nhwc(x, ws[i], ci, 1, 1, bias=b, residual=kw.get("residual"),
                                             out=outs[i], amax=a)
            hot = graph_us([mk(0)] * NW)
            cold = graph_us([mk(i) for i in range(NW)])
            rows.append(f"{label} {hot:.1f} / {cold:.1f}")
        fl = 2.0 * n * h * h * co * 9 * ci
        print(f"conv {n}x{h}x{h} {ci}->{co}: us hot / cold weights: " + " | ".join(rows) + f"  ({fl / 1e9:.1f} GFLOP)",
              flush=True)


if __name__ == "__main__":
    main()
