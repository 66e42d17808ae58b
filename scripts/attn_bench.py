"""Attention kernel timing on the path's shapes (HIP events), for configuration sweeps:
python scripts/attn_bench.py [cfg]   (cfg: qd_attn_force - 1|2|3|5|6 k_attn, 7|8 k_attn32 waves)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import _lib
from qdiff import kernels as K

dev = "cuda:0"
CFG = int(sys.argv[1]) if len(sys.argv) > 1 else 0
_lib.load().qd_attn_force(CFG)
for (b, s, skv, heads, d, ld) in ((8, 4096, 4096, 8, 40, 960), (8, 1024, 1024, 10, 64, 1920), (2, 4429, 4429, 38, 64, 7296),
                                  (8, 4096, 77, 8, 40, 320), (8, 1024, 1024, 8, 80, 1920), (8, 256, 256, 8, 160, 3840),
                                  (4, 4096, 4096, 10, 64, 1920), (4, 1024, 1024, 20, 64, 3840),
                                  (8, 1024, 77, 8, 80, 640), (8, 256, 77, 8, 160, 1280), (8, 64, 77, 8, 160, 1280)):
    c = heads * d
    x = torch.randn(b, s, ld, device=dev).half()
    kv = torch.randn(b, skv, ld, device=dev).half()
    q, k, v = x[:, :, :c], kv[:, :, c:2 * c] if ld >= 2 * c else kv[:, :, :c], kv[:, :, ld - c:]
    for _ in range(3):
        K.attention(q, k, v, heads)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        K.attention(q, k, v, heads)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    fl = 4.0 * b * heads * s * skv * d
    print(f"cfg={CFG or '-'} b={b} sq={s} skv={skv} h={heads} d={d}: {us:.1f} us  {fl / us / 1e6:.0f} TFLOP/s", flush=True)
