"""GEGLU projection GEMMs of the SD1.5 levels (CFG batch 8): tuned time and every forced variant,
fp16 weights and int8 codes, with the fused GEGLU epilogue and with a plain epilogue (same MFMA
work, 2x the output bytes, no GELU) - how much of the launch the GELU VALU costs.
usage: python scripts/geglu_sweep.py"""
import os
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
    g = torch.Generator(device="cpu").manual_seed(0)
    for (m, n, k) in ((32768, 2560, 320), (8192, 5120, 640), (2048, 10240, 1280)):
        x = torch.randn(m, k, generator=g).half().to(dev)
        w = (torch.randn(n, k, generator=g) / k ** 0.5).half().to(dev)
        b = torch.randn(n, generator=g).half().to(dev)
        perm = K.geglu_interleave_rows(n, dev)
        wg, bg = w[perm].contiguous(), b[perm].contiguous()
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(wg, k, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()
        res = {}
        for label, fn in (("f16 geglu", lambda: K.linear(x, wg, "f16", bias=bg, geglu=True)),
                          ("f16 plain", lambda: K.linear(x, wg, "f16", bias=bg)),
                          ("i8 geglu", lambda: K.linear_i8(xq, sa, wq, sw, bias=bg, geglu=True)),
                          ("i8 plain", lambda: K.linear_i8(xq, sa, wq, sw, bias=bg))):
            res[label] = timeit(fn)
        print(f"M {m} N {n} K {k}: " + " | ".join(f"{kk} {v:.1f} us" for kk, v in res.items()), flush=True)
        for label, vs, fn in (("f16 geglu", K.REG_VARIANTS + K.DMA_VARIANTS,
                               lambda: K.linear(x, wg, "f16", bias=bg, geglu=True)),
                              ("i8 geglu", K.I8_VARIANTS, lambda: K.linear_i8(xq, sa, wq, sw, bias=bg, geglu=True))):
            row = []
            for v in vs:
                K.force_gemm(v)
                try:
                    row.append(f"{v}:{timeit(fn):.1f}")
                except Exception:  # noqa: BLE001
                    row.append(f"{v}:x")
                K.force_gemm(None)
            print(f"    {label} forced: " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
