"""Save attention outputs of the path's shapes under the current QD_ATTN_CFG (compare two
configurations bit for bit): python scripts/attn_cmp.py OUT.pt | python scripts/attn_cmp.py --diff A.pt B.pt"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

if sys.argv[1] == "--diff":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for k in a:
        same = torch.equal(a[k], b[k])
        print(k, "bit-identical" if same else f"DIFFER max {float((a[k].float() - b[k].float()).abs().max()):.3g}")
    sys.exit(0)
import qdiff_boot  # noqa
from qdiff import kernels as K

out = {}
for (b, s, skv, heads, d) in ((8, 4096, 4096, 8, 40), (2, 1000, 1000, 8, 40), (4, 4096, 333, 8, 40),
                              (8, 1024, 1024, 10, 64), (2, 777, 777, 5, 64), (8, 1024, 1024, 8, 80)):
    g = torch.Generator().manual_seed(s + d)
    c = heads * d
    q = torch.randn(b, s, c, generator=g).half().cuda()
    k = torch.randn(b, skv, c, generator=g).half().cuda()
    v = torch.randn(b, skv, c, generator=g).half().cuda()
    out[f"{b}x{s}x{skv}x{heads}x{d}"] = K.attention(q, k, v, heads).cpu()
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])
