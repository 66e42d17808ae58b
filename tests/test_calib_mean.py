"""SmoothQuant statistics over calls: the reference averages each hooked linear's
per-call channel maxima with mean_of_dict (/root/reference/models/StableDiffusion1_x.py:104-112 =
torch.mean of the stacked fp16 vectors) after Mean_Max_Activation_Hook recorded them
(utils/calib_data.py:105-124).  tests/golden/make_golden.py ran both reference functions over 3, 24
and 600 calls (600 = the reference's calibration: 12 pipeline calls x 50 steps), with magnitudes
spread over ~2^14 so the fp32 sums round; calib.MeanMaxActivationHook must give the same fp16 bits.
The goldens ran on CPU tensors, so what is pinned is torch's CPU reduction order; the reference's
own calibration runs on CUDA (utils/calib_data.py:235), whose torch.mean order is not pinned here."""
import numpy as np
import pytest
import torch

from qdiff.calib import MeanMaxActivationHook

CALLS = (3, 24, 600)


@pytest.mark.parametrize("calls", CALLS)
def test_hook_mean_matches_reference_mean_of_dict(golden, calls):
    g = golden["smooth_golden"]
    xs = g[f"mean{calls}_x"]                     # [calls, 1, rows, C] fp16
    want = g[f"mean{calls}_mean"]
    hook = MeanMaxActivationHook(xs.shape[-1], "cpu")
    for xi in xs:
        # the per-call reduction (calib_data.py:111-112): max |x| per channel over the rows, fp16
        hook.record_max(torch.from_numpy(xi.reshape(-1, xi.shape[-1])).abs().amax(0))
    got = hook.mean().numpy()
    assert got.dtype == np.float16 and np.array_equal(got.view(np.uint16), want.view(np.uint16)), \
        (got != want).sum()
    # the inputs do exercise the summation order: the cascade's fp32 sums differ from a plain
    # sequential fp32 sum in some channels (before the fp16 rounding of the mean hides most of it)
    seq = np.zeros(xs.shape[-1], np.float32)
    for xi in xs:
        seq += np.abs(xi.reshape(-1, xi.shape[-1]).astype(np.float32)).max(0)
    tot = sum(a for a in hook.acc[1:]) + hook.acc[0]
    if calls >= 24:
        assert not np.array_equal(tot.numpy(), seq)


@pytest.mark.gpu
@pytest.mark.parametrize("calls", CALLS)
def test_gpu_hook_mean_matches_reference_mean_of_dict(golden, dev, calls):
    """The same through the product hook's device path (qd_channel_absmax_accum per call)."""
    g = golden["smooth_golden"]
    xs = g[f"mean{calls}_x"]
    hook = MeanMaxActivationHook(xs.shape[-1], dev)
    for xi in xs:
        hook(torch.from_numpy(np.ascontiguousarray(xi.reshape(-1, xi.shape[-1]))).to(dev))
    got = hook.mean().cpu().numpy()
    assert np.array_equal(got.view(np.uint16), g[f"mean{calls}_mean"].view(np.uint16))
