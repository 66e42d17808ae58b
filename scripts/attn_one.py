"""One attention shape, a few launches (profiling driver): python scripts/attn_one.py [d] [iters] [cfg]
d = 40 (SD1.5 64x64 level self-attention, b 8, 8 heads, 4096 tokens) or 64 (SD3.5-L joint, b 2, 38 heads)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import _lib
from qdiff import kernels as K

d = int(sys.argv[1]) if len(sys.argv) > 1 else 40
it = int(sys.argv[2]) if len(sys.argv) > 2 else 5
_lib.load().qd_attn_force(int(sys.argv[3]) if len(sys.argv) > 3 else 0)  # (cfg: the kernel choice knob)
b, s, heads, ld = (8, 4096, 8, 960) if d == 40 else (2, 4429, 38, 7296)
c = heads * d
x = torch.randn(b, s, ld, device="cuda:0").half()
q, k, v = x[:, :, :c], x[:, :, c:2 * c], x[:, :, 2 * c:3 * c]
for _ in range(it):
    K.attention(q, k, v, heads)
torch.cuda.synchronize()
print("ok")
