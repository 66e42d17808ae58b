"""Short-K linears of the SD1.5 64x64 / 32x32 levels (N = C, K = C): tuned time and every forced
variant, int8 and fp16, with and without the residual add, next to copy kernels that move the same
HBM bytes (the practical floor).  --pmc: run only the tuned int8 M 32768 N 320 K 320 + residual
shape a few times (profiling driver).
usage: python scripts/shortk_i8.py [--iters 20] [--pmc]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def operands(m, c, dev, g):
    x = torch.randn(m, c, generator=g).half().to(dev)
    w = (torch.randn(c, c, generator=g) / c ** 0.5).half().to(dev)
    r = torch.randn(m, c, generator=g).half().to(dev)
    xq, sa = K.quant_rows_i8(x)
    wq, sw16, _ = K.weight_quant(w, c, 8, want_dq=False)
    return x, w, r, xq, sa, wq, sw16.float().view(-1).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pmc", action="store_true")
    ap.add_argument("--pmc-n", type=int, default=320,
                    help="--pmc: N of the M 32768 K 320 int8 linear (2560: the plain wide-N shape, no residual)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    if a.pmc and a.pmc_n != 320:
        x = torch.randn(32768, 320, generator=g).half().to(dev)
        w = (torch.randn(a.pmc_n, 320, generator=g) / 320 ** 0.5).half().to(dev)
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(w, 320, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()
        b = torch.randn(a.pmc_n, generator=g).half().to(dev)
        for _ in range(5):
            K.linear_i8(xq, sa, wq, sw, bias=b)
        torch.cuda.synchronize()
        print("choice", [v for kk, v in K.gemm_choices(used_only=True).items()])
        return
    if a.pmc:
        x, w, r, xq, sa, wq, sw = operands(32768, 320, dev, g)
        for _ in range(5):
            K.linear_i8(xq, sa, wq, sw, residual=r)
        torch.cuda.synchronize()
        print("choice", [v for kk, v in K.gemm_choices(used_only=True).items()])
        return
    for (m, c) in ((32768, 320), (8192, 640)):
        x, w, r, xq, sa, wq, sw = operands(m, c, dev, g)
        out = torch.empty(m, c, dtype=torch.float16, device=dev)
        # copy floors: read A (fp16 / int8) + write out (+ read residual)
        t_cp16 = timeit(lambda: out.copy_(x), a.iters)
        t_cp16r = timeit(lambda: torch.add(x, r, out=out), a.iters)
        x8 = xq.view(torch.uint8)
        t_cp8 = timeit(lambda: out.copy_(x8), a.iters)
        print(f"M {m} C {c}: copy f16->f16 {t_cp16:.1f} us, add f16+f16->f16 {t_cp16r:.1f} us, "
              f"u8->f16 {t_cp8:.1f} us", flush=True)
        for res in (False, True):
            rr = r if res else None
            ti = timeit(lambda: K.linear_i8(xq, sa, wq, sw, residual=rr), a.iters)
            tf = timeit(lambda: K.linear(x, w, "f16", residual=rr), a.iters)
            ch = [v for kk, v in K.gemm_choices(used_only=True).items() if kk[1:4] == (m, c, c)]
            hbm_i8 = m * c * (1 + 2 + (2 if res else 0))
            hbm_f16 = m * c * (2 + 2 + (2 if res else 0))
            print(f"  residual={res}: int8 {ti:.1f} us ({hbm_i8 / ti / 1e3:.0f} GB/s) | fp16 {tf:.1f} us "
                  f"({hbm_f16 / tf / 1e3:.0f} GB/s)  choices {ch}", flush=True)
            row = []
            for v in K.I8_VARIANTS:
                K.force_gemm(v)
                try:
                    row.append(f"{v}:{timeit(lambda: K.linear_i8(xq, sa, wq, sw, residual=rr), a.iters):.1f}")
                except Exception as e:  # noqa: BLE001
                    row.append(f"{v}:x")
                K.force_gemm(None)
            print("    int8 forced:", " ".join(row), flush=True)
            row = []
            for v in K.REG_VARIANTS + K.DMA_VARIANTS:
                K.force_gemm(v)
                try:
                    row.append(f"{v}:{timeit(lambda: K.linear(x, w, 'f16', residual=rr), a.iters):.1f}")
                except Exception as e:  # noqa: BLE001
                    row.append(f"{v}:x")
                K.force_gemm(None)
            print("    fp16 forced:", " ".join(row), flush=True)


if __name__ == "__main__":
    main()
