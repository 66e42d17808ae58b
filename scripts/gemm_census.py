"""Per-shape GEMM census of one SD1.5 W8A8 UNet eval (CFG batch 8): every linear / conv call,
its tuned kernel choice and its HIP-event time (eager, after tuning).
usage: python scripts/gemm_census.py [--int8]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402
from qdiff.models import StableDiffusion1_x  # noqa: E402
from qdiff.pipeline import synthetic_text_embeddings  # noqa: E402

dev = torch.device("cuda:0")
model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
INT8 = "--int8" in sys.argv
model.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True,
               int8_mfma=INT8)
loop = model.get_loop(4, 512, 512, 50, 7.5, use_graph=False)
ctx = torch.cat([synthetic_text_embeddings([""] * 4, device=dev), synthetic_text_embeddings([f"p{i}" for i in range(4)], device=dev)])
lat = torch.randn(4, 4, 64, 64, generator=torch.Generator().manual_seed(0)).half().to(dev)
loop.set_inputs(lat, ctx)
loop.step()  # tunes every shape
torch.cuda.synchronize()
rec = collections.defaultdict(list)
orig_lin, orig_conv = K.linear, K.conv2d_nhwc
orig_lin8, orig_conv8 = K.linear_i8, K.conv2d_i8


def timed(kind, fn):
    def w(*a, **k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn(*a, **k)
        e1.record()
        x = a[0]
        if kind == "linear_i8":
            key = (kind, x.shape[0], a[2].shape[0], x.shape[1], "geglu" if k.get("geglu") else "")
            fl = 2 * x.shape[0] * a[2].shape[0] * x.shape[1]
        elif kind == "conv_i8":
            wt = a[2]
            key = (kind, tuple(x.shape), wt.shape[0], a[4], "ups" if (len(a) > 7 and a[7]) else "")
            fl = 2 * out.numel() * wt[0].numel()
        elif kind == "linear":
            key = (kind, x.shape[0], a[1].shape[0], x.shape[1], "geglu" if k.get("geglu") else "")
            fl = 2 * x.shape[0] * a[1].shape[0] * x.shape[1]
        else:
            wt = a[1]
            key = (kind, tuple(x.shape), wt.shape[0], wt.shape[1], "ups" if (len(a) > 5 and a[5]) or k.get("upsample2x") else "")
            fl = 2 * out.numel() * wt[0].numel()
        rec[key].append((e0, e1, fl))
        return out
    return w


K.linear, K.conv2d_nhwc = timed("linear", orig_lin), timed("conv", orig_conv)
K.linear_i8, K.conv2d_i8 = timed("linear_i8", orig_lin8), timed("conv_i8", orig_conv8)
import qdiff.unet as U  # noqa: E402
loop.step()
torch.cuda.synchronize()
rows = []
for key, v in rec.items():
    t = sum(e0.elapsed_time(e1) for e0, e1, _ in v) * 1e3
    fl = sum(f for _, _, f in v)
    rows.append((t, key, len(v), fl / t / 1e6))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"GEMM total {tot / 1e3:.3f} ms per eval (eager, event-timed incl. launch gaps)")
for t, key, n, tf in rows:
    print(f"{t:8.1f} us  x{n:2d}  {tf:6.0f} TF/s  {key}")
print("choices:")
for k, c in K.gemm_choices().items():
    print(" ", k, "->", c)
