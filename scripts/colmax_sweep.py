"""k_colmax_nhwc launch-geometry sweep: python scripts/colmax_sweep.py MIN_BLOCKS MAX_ROWS_PER_THREAD
(qd_colmax_geom_force; one process per setting under rocprofv3)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import _lib
from qdiff import kernels as K

dev = "cuda:0"
MINBLK, MAXRPT = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (0, 0)
_lib.load().qd_colmax_geom_force(MINBLK, MAXRPT)
res = []
for shp in ((8, 64, 64, 320), (8, 32, 32, 640), (8, 16, 16, 1280), (8, 8, 8, 1280), (8, 64, 64, 640)):
    x = torch.randn(*shp, device=dev).half()
    for _ in range(3):
        K.act_absmax(x, "per_channel", K.NHWC)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        K.act_absmax(x, "per_channel", K.NHWC)
    e1.record(); e1.synchronize()
    res.append(f"{shp}:{e0.elapsed_time(e1) / 50 * 1e3:.1f}")
print(MINBLK, MAXRPT, " ".join(res), flush=True)
