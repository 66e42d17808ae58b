"""Print bench.py's dominant-conv roofline objects (both modes) - a quick check of their avg_us against
the step sequences' durations of the same launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
import bench  # noqa: E402

dev = torch.device("cuda:0")
for mb in (0, 64, 128, 512):
    bench.ROOF_FLUSH_MB = mb
    for i8 in (False, True):
        r = bench.dominant_kernel_roofline(dev, int8=i8)
        print(f"flush {mb} MB", ("int8" if i8 else "fp16"), r["avg_us"], r["achieved"], r["frac"], flush=True)
