"""Diagnostic: the halo conv (variant 200) on the SD1.5 64x64 320->320 shape with each
scripts/ablate/libqdiff_abl<bits>.so (scripts/halo_ablate.sh) - which part of its K loop costs what.
usage: python scripts/halo_ablate.py <bits> [<bits> ...]   (0 = the in-tree library)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 or (len(sys.argv) == 2 and sys.argv[1] == "all"):
    bits = sys.argv[1:] if sys.argv[1] != "all" else ["0", "1", "2", "4", "6", "8", "14", "15"]
    for b in bits:  # one process per library (each loads its own libqdiff)
        subprocess.run([sys.executable, __file__, b], check=True)
    sys.exit(0)
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import _lib  # noqa: E402

b = sys.argv[1]
if b != "0":
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "ablate", f"libqdiff_abl{b}.so")
from qdiff import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn(8, 64, 64, 320, device=dev).half()
wt = (torch.randn(320, 3, 3, 320, device=dev) * 0.02).half()
bias = torch.zeros(320, device=dev).half()
am = torch.empty(8 * 320, device=dev)
var = int(os.environ.get("QD_HALO_VAR", "200"))
K.force_gemm(var)
if var >= 140:  # the int8 halo conv (int8-MFMA mode) on the same shape
    xq, sa = K.quant_samples_i8(x)
    wq, sw16, _ = K.weight_quant(wt.view(320, -1).contiguous(), 9 * 320, 8, want_dq=False)
    wq, sw = wq.view(320, 3, 3, 320), sw16.float().view(-1).contiguous()
    fn = lambda: K.conv2d_i8(xq, sa, wq, sw, 320, 1, 1, bias=bias)  # noqa: E731
else:
    fn = lambda: K.conv2d_nhwc(x, wt, 320, 1, 1, bias=bias, amax=am)  # noqa: E731
for _ in range(5):
    fn()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
print(f"var {var} abl {b:>2}: {min(ts):7.1f} us", flush=True)
