"""GroupNorm chain geometry sweep on the SD1.5 CFG-batch-8 shapes (HIP-event timed, back-to-back
launches): the GN-fin form (statistics pass materialising x = half(fq(y) + residual)), the
fused-temb form and the plain GroupNorm(+SiLU)+fake-quant, for rows-per-thread settings of the
statistics / apply passes (qd_gn_geom_force).

usage: python scripts/gn_bench.py [--sweep]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import _lib  # noqa: E402
from qdiff import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, iters=30, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream()
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


SHAPES = [(8, 4096, 320), (8, 4096, 640), (8, 1024, 640), (8, 1024, 1280)]


def run(settings):
    lib = _lib.load()
    for n, hw, c in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        y = torch.randn(n, hw, c, device=dev, generator=g).half()
        res = torch.randn(n, hw, c, device=dev, generator=g).half()
        amax = y.float().abs().amax(dim=1).reshape(-1).contiguous()
        temb = torch.randn(n, c, device=dev, generator=g).half()
        gam = (1 + 0.1 * torch.randn(c, device=dev, generator=g)).half()
        bet = (0.1 * torch.randn(c, device=dev, generator=g)).half()
        mb = n * hw * c * 2 / 1e6
        ref = None
        for srpt, arpt in settings:
            lib.qd_gn_geom_force(srpt, arpt)
            fin = lambda: K.groupnorm_fin(y, amax, 8, res, 32, 1e-5, gam, bet, silu=True, q_bits=8)
            tmb = lambda: K.groupnorm_fin(y, amax, 8, None, 32, 1e-5, gam, bet, silu=True, q_bits=8, cadd=temb)
            pln = lambda: K.groupnorm_nhwc(res, 32, 1e-5, gam, bet, silu=True, q_bits=8)
            out = fin()
            if ref is None:
                ref = out
            same = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
            tf, tt, tp = timeit(fin), timeit(tmb), timeit(pln)
            print(f"n={n} hw={hw:5d} c={c:5d} srpt={srpt:2d} arpt={arpt:2d}: fin {tf:6.1f} us "
                  f"({5 * mb / tf * 1e-3:5.2f} TB/s)  temb {tt:6.1f} us  plain {tp:6.1f} us "
                  f"({3 * mb / tp * 1e-3:5.2f} TB/s)  same-as-first {same}", flush=True)
    lib.qd_gn_geom_force(0, 0)


SMALL = [(8, 256, 640), (8, 256, 1280), (8, 256, 1920), (8, 64, 1280), (8, 64, 2560), (8, 256, 960)]


def run_small():
    """The single-kernel GroupNorm (hw <= 256): plain GroupNorm + SiLU + fake-quant, and the fq_in form
    (the conv output's fake-quant + temb add recomputed on the fly)."""
    for n, hw, c in SMALL:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(n, hw, c, device=dev, generator=g).half()
        amax = x.float().abs().amax(dim=1).reshape(-1).contiguous()
        temb = torch.randn(n, c, device=dev, generator=g).half()
        gam = (1 + 0.1 * torch.randn(c, device=dev, generator=g)).half()
        bet = (0.1 * torch.randn(c, device=dev, generator=g)).half()
        pln = lambda: K.groupnorm_nhwc(x, 32, 1e-5, gam, bet, silu=True, q_bits=8)
        fqi = lambda: K.groupnorm_nhwc(x, 32, 1e-5, gam, bet, silu=True, q_bits=8, fq_in=(amax, 8, temb))
        print(f"small n={n} hw={hw:4d} c={c:5d}: plain {timeit(pln):6.1f} us  fq_in+temb {timeit(fqi):6.1f} us",
              flush=True)


if __name__ == "__main__":
    if "--small" in sys.argv:
        run_small()
        sys.exit(0)
    if "--sweep" in sys.argv:
        run([(0, 0)] + [(s, a) for s in (4, 8, 16, 32) for a in (2, 4, 8, 16)])
    elif "--srpt" in sys.argv:  # statistics-pass rows per thread only (apply pass at its rule)
        run([(0, 0)] + [(s, 0) for s in (2, 4, 8, 16, 32)])
    else:
        run([(0, 0)])
