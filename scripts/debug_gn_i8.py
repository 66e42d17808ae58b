"""Locate the elements where the fused int8 GroupNorm codes differ from the per-sample codes of
the fp16 GroupNorm output (tests/test_gpu_int8.py::test_groupnorm_i8_equals_quantized_groupnorm)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import qdiff_boot  # noqa
from qdiff import kernels as k

dev = "cuda:0"
for silu in (False, True):
    for hw in (16, 32):
        g = torch.Generator().manual_seed(5)
        n, h, w, c1 = 2, hw, hw, 320
        x = (torch.randn(n, h, w, c1, generator=g) * 3).half().to(dev)
        c = c1
        gamma = (1 + 0.1 * torch.randn(c, generator=g)).half().to(dev)
        beta = (0.1 * torch.randn(c, generator=g)).half().to(dev)
        ref16 = k.groupnorm_nhwc(x, 32, 1e-5, gamma, beta, silu=silu)
        q_ref, s_ref = k.quant_samples_i8(ref16)
        q, s = k.groupnorm_nhwc_i8(x, 32, 1e-5, gamma, beta, silu=silu)
        bad = (q != q_ref).nonzero()
        print(f"silu={silu} hw={hw}: scales equal {torch.equal(s, s_ref)}, {bad.shape[0]} code mismatches")
        for b in bad[:6].tolist():
            v = ref16[tuple(b)].item()
            print("   at", b, "ref16", v, "v/s", v / s[b[0]].item(), "codes", q[tuple(b)].item(), q_ref[tuple(b)].item())
