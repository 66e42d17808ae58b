"""HBM-bound pass timings on the SD1.5 64x64-level tensor ([8, 64, 64, 320] fp16, 21 MB), graph-timed,
next to a plain copy and add (the achievable floor at this size)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import kernels as K
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from shape_bench import graph_time  # noqa: E402

dev = "cuda:0"
g = torch.Generator().manual_seed(0)
for (n, h, w, c) in ((8, 64, 64, 320), (8, 32, 32, 640), (8, 16, 16, 1280)):
    x = torch.randn(n, h, w, c, generator=g).half().to(dev)
    r = torch.randn(n, h, w, c, generator=g).half().to(dev)
    y = torch.empty_like(x)
    amax = (x.float().abs().amax(dim=(1, 2)) * 1.01).reshape(-1).contiguous()
    gam = torch.ones(c, dtype=torch.float16, device=dev)
    bet = torch.zeros(c, dtype=torch.float16, device=dev)
    mb = x.numel() * 2 / 1e6
    rows = [
        ("copy (torch)", lambda: y.copy_(x), 2),
        ("add (qd_add)", lambda: K.add(x, r, out=y), 3),
        ("finalize fq+res", lambda: K.fq_finalize(x, amax, 8, residual=r, out=y), 3),
        ("act_absmax per-ch", lambda: K.act_absmax(x, "per_channel", K.NHWC), 1),
        ("act_apply per-ch", lambda: K.act_apply_nhwc(x, amax, 8, out=y), 2),
        ("layernorm", lambda: K.layernorm(x.view(-1, c), 1e-5, gam, bet, out=y.view(-1, c)), 2),
        ("finalize+layernorm", lambda: K.layernorm(K.fq_finalize(x, amax, 8, out=r).view(-1, c), 1e-5, gam, bet,
                                                   out=y.view(-1, c)), 5),
        ("layernorm_fq", lambda: K.layernorm_fq(x.view(-1, c), amax, 8, h * w, 1e-5, gam, bet), 3),
        ("groupnorm+silu+fq", lambda: K.groupnorm_nhwc(x, 32, 1e-5, gam, bet, silu=True, q_bits=8, out=y), 3),
        ("groupnorm", lambda: K.groupnorm_nhwc(x, 32, 1e-5, gam, bet, out=y), 3),
        ("gn+silu+fq fq_in", lambda: K.groupnorm_nhwc(x, 32, 1e-5, gam, bet, silu=True, q_bits=8, out=y,
                                                    fq_in=(amax, 8, None)), 3),
        ("gn+silu+fq fin", lambda: K.groupnorm_fin(x, amax, 8, None, 32, 1e-5, gam, bet, silu=True, q_bits=8), 4),
        ("gn+silu+fq fin+res", lambda: K.groupnorm_fin(x, amax, 8, r, 32, 1e-5, gam, bet, silu=True, q_bits=8), 5),
    ]
    print(f"[{n},{h},{w},{c}] {mb:.1f} MB per tensor")
    for name, fn, passes in rows:
        us = graph_time(fn, 20)
        print(f"  {name:20s} {us:7.1f} us  {passes * mb / us:5.2f} TB/s ({passes} tensor passes)", flush=True)
