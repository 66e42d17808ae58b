"""int8 linears at SD1.5's short-K shapes: every LDS-DMA / ping-pong variant against the persistent
ones (qd_gemm_force 160+ / 170+), HIP-event timed in one process, outputs checked bit-equal to the
one-tile variant's.  usage: python scripts/persist_sweep.py"""
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


def main_f16():
    """fp16 linears (the fake-quant mode's operands): the one-tile variants vs persistent ones (ids 420 + v
    were a round-5 build's persistent fp16 tiles: no faster anywhere, profiles/r05q_sweep_f16.log; the
    current library rejects them, so they drop out of this sweep)."""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    shapes = [(32768, 320, 320, "res"), (32768, 960, 320, "plain"), (32768, 320, 320, "plain"),
              (8192, 640, 640, "res"), (8192, 1920, 640, "plain"), (2048, 1280, 1280, "res"),
              (2048, 3840, 1280, "plain"), (32768, 320, 1280, "res"), (8192, 5120, 640, "geglu")]
    for M, N, Kd, epi in shapes:
        x = torch.randn(M, Kd, generator=g).half().to(dev)
        w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(dev)
        b = torch.randn(N, generator=g).half().to(dev)
        r = torch.randn(M, N, generator=g).half().to(dev) if epi == "res" else None

        def run():
            return K.linear(x, w, "f16", bias=b, residual=r, geglu=epi == "geglu")
        K.force_gemm(100)
        ref = run().clone()
        res = []
        for v in list(K.REG_VARIANTS) + list(K.DMA_VARIANTS) + [420, 422, 424, 430, 431, 436, 437]:
            K.force_gemm(v)
            try:
                y = run()
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            same = torch.equal(y.view(torch.int16), ref.view(torch.int16))
            t = statistics.median([timeit(run) for _ in range(3)])
            res.append((t, v, same))
        K.force_gemm(None)
        res.sort()
        line = "  ".join(f"{v}:{t:.1f}{'' if ok else '!MISMATCH'}" for t, v, ok in res[:8])
        bad = [v for _, v, ok in res if not ok]
        print(f"f16 M{M} N{N} K{Kd} {epi:5s} best {line}" + (f"   MISMATCH {bad}" if bad else ""), flush=True)


def main():
    if "--f16" in sys.argv:
        return main_f16()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    shapes = [(32768, 320, 320, "res"), (32768, 960, 320, "plain"), (32768, 320, 320, "plain"),
              (8192, 640, 640, "res"), (8192, 1920, 640, "plain"), (2048, 1280, 1280, "res"),
              (32768, 320, 1280, "res"), (8192, 5120, 640, "geglu"), (32768, 2560, 320, "plain"),
              (32768, 960, 320, "bias"), (8192, 1920, 640, "plain"), (32768, 2560, 320, "geglu")]
    for M, N, Kd, epi in shapes:
        x = torch.randn(M, Kd, generator=g).half().to(dev)
        w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(dev)
        b = torch.randn(N, generator=g).half().to(dev) if epi != "plain" else None
        r = torch.randn(M, N, generator=g).half().to(dev) if epi == "res" else None
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(w, Kd, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()

        def run():
            return K.linear_i8(xq, sa, wq, sw, bias=b, residual=r, geglu=epi == "geglu")
        K.force_gemm(110)
        ref = run().clone()
        res = []
        for v in list(K.I8_VARIANTS) + list(K.I8_PERSIST_VARIANTS) + list(K.I8_AS_VARIANTS):
            K.force_gemm(v)
            try:
                y = run()
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            same = torch.equal(y.view(torch.int16), ref.view(torch.int16))
            t = statistics.median([timeit(run) for _ in range(3)])
            res.append((t, v, same))
        K.force_gemm(None)
        res.sort()
        line = "  ".join(f"{v}:{t:.1f}{'' if ok else '!MISMATCH'}" for t, v, ok in res[:8])
        bad = [v for _, v, ok in res if not ok]
        print(f"M{M} N{N} K{Kd} {epi:5s} best {line}" + (f"   MISMATCH {bad}" if bad else ""), flush=True)


if __name__ == "__main__":
    main()
