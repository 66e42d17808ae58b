"""GEGLU epilogue ablation on the SD1.5 64x64-level feed-forward projection (M 32768, K 320, N 2560
-> 1280 outputs) and the 32x32 one (M 8192, K 640, N 5120): per fp16 variant, the GEGLU launch vs the
same GEMM with a plain fp16 output (N columns, twice the stores) and vs half the columns (N / 2, the
GEGLU output's store volume), warm (graph replay) and cold (512 MB flush before each launch).

usage: python scripts/geglu_ablate.py [--variants 17 13 ...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from epi_ablate import cold_time, warm_time  # noqa: E402

dev = torch.device("cuda:0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="*", type=int, default=[])
    a = ap.parse_args()
    variants = [None] + (a.variants or list(K.DMA_VARIANTS))
    g = torch.Generator(device="cpu").manual_seed(0)
    for (m, n, k) in [(32768, 2560, 320), (8192, 5120, 640)]:
        x = torch.randn(m, k, generator=g).half().to(dev)
        w = (torch.randn(n, k, generator=g) / k ** 0.5).half().to(dev)
        b = (0.1 * torch.randn(n, generator=g)).half().to(dev)
        wh, bh = w[: n // 2].contiguous(), b[: n // 2].contiguous()
        forms = {
            "geglu": lambda: K.linear(x, w, bias=b, geglu=True),
            "plain N": lambda: K.linear(x, w, bias=b),
            "plain N/2": lambda: K.linear(x, wh, bias=bh),
        }
        print(f"M {m} N {n} K {k}: {2.0 * m * n * k / 1e9:.1f} GFLOP", flush=True)
        for name, fn in forms.items():
            cells = []
            for v in variants:
                K.force_gemm(v)
                try:
                    cells.append(f"{v}:{warm_time(fn):.1f}/{cold_time(fn):.1f}")
                except RuntimeError:
                    cells.append(f"{v}:err")
                finally:
                    K.force_gemm(None)
            print(f"  {name:10s} warm/cold us  " + " ".join(cells), flush=True)


if __name__ == "__main__":
    main()
