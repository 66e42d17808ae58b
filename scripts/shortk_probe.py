"""Short-K GEMM probe (SD1.5 64x64-level linears, M = 32768): the tuned libqdiff time vs K
(320 / 640 / 1280) and vs the epilogue (GEGLU, plain), next to torch.matmul, graph-timed.
Separates the per-tile fixed cost (pipeline fill + epilogue) from the K loop."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from shape_bench import graph_time  # noqa: E402

dev = "cuda:0"
for (m, n, geglu) in ((32768, 2560, True), (32768, 2560, False), (32768, 960, False), (32768, 320, False)):
    for k in (320, 640, 1280):
        a = torch.randn(m, k, device=dev).half()
        w = (torch.randn(n, k, device=dev) / k ** 0.5).half()
        b = torch.randn(n, device=dev).half()
        K.linear(a, w, "f16", bias=b, geglu=geglu)  # tune
        us = graph_time(lambda: K.linear(a, w, "f16", bias=b, geglu=geglu), 20)
        ref = graph_time(lambda: torch.matmul(a, w.t()), 20)
        ch = K.gemm_choices()
        fl = 2.0 * m * n * k
        print(f"M={m} N={n} K={k} geglu={geglu}: {us:7.1f} us ({fl / us / 1e6:5.0f} TF/s)  matmul {ref:7.1f} us  "
              f"choice {list(ch.values())[-1] if ch else '-'}", flush=True)
