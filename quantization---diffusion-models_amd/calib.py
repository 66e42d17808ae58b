"""SmoothQuant calibration: per-channel activation absmax hooks and the calibration run.

``MeanMaxActivationHook`` is utils/calib_data.py:105-124 (Mean_Max_Activation_Hook): on every
forward call of a Linear it records max |x| per input channel; the adapter later averages the
per-call vectors (StableDiffusion1_x.py:104-112, mean_of_dict).  Here the per-call reduction is
the wavefront-shuffle kernel ``qd_channel_absmax_accum`` and the running sum stays on device.

The fused UNet forward calls Linear layers through ``unet.run_linear`` (not nn.Module
__call__), so hooks are attached as a ``_qd_hook`` attribute that run_linear invokes.

Calibration data: the reference streams 96 COCO captions (network; unavailable offline) and
draws latents randn(8, 4, 64, 64) from torch.manual_seed(42) (calib_data.py:174-213), then runs
12 pipeline calls x 50 steps at CFG 7.5 (:227-245).  ``synthetic_calibration_set`` keeps the
seed / batch / latent recipe and replaces the captions with deterministic synthetic prompts.
"""
import torch
from torch import nn

from . import kernels as K


# torch's CPU sum over the stacked calls (mean_of_dict -> torch.mean of fp16 = fp32 sum / count ->
# fp16) accumulates rows in the multi-level cascade of aten/src/ATen/native/cpu/SumKernel.cpp
# (multi_row_sum): 16 rows into level 0, then level j += level j-1 whenever the row count is a
# multiple of 16^j, the levels added 0 += 1 += 2 += 3 at the end (level width 16 while the call
# count is <= 2^16).  The hook keeps the same four fp32 accumulators on device, so mean() has the
# bits of the reference's mean_of_dict over CPU tensors (tests/test_calib_mean.py pins that CPU
# reduction order).  The reference calibrates on CUDA (utils/calib_data.py:235), where torch.mean
# reduces in the device's own order: parity with that run is to within fp32 rounding of the sum,
# i.e. unpinned at the bit level.
_LEVEL_BITS, _LEVELS, _MAX_CALLS = 4, 4, 1 << 16


class MeanMaxActivationHook:
    def __init__(self, channels, device):
        # acc[0] (= self.sum) receives each call's per-channel max; acc[1..3] the cascade levels
        self.acc = [torch.zeros(channels, dtype=torch.float32, device=device) for _ in range(_LEVELS)]
        self.ws = torch.empty(channels, dtype=torch.float32, device=device)
        self.count = 0
        self.hook_handle = None

    @property
    def sum(self):
        return self.acc[0]

    def __call__(self, x2d):
        K.channel_absmax_accum(x2d, self.ws, self.acc[0])
        self._advance()

    def record_max(self, amax):
        """One call's per-channel max |x| (fp16 or fp32 values), accumulated like __call__."""
        self.acc[0] += amax.to(torch.float32)
        self._advance()

    def _advance(self):
        self.count += 1
        i = self.count
        if i % (1 << _LEVEL_BITS):
            return
        for j in range(1, _LEVELS):  # a full 16-row chunk: carry level j-1 into level j
            self.acc[j] += self.acc[j - 1]
            self.acc[j - 1].zero_()
            if i & (((1 << _LEVEL_BITS) - 1) << (j * _LEVEL_BITS)):
                break

    def mean(self):
        """mean over recorded calls with the reference's bits: fp32 cascade sum / count -> fp16
        (StableDiffusion1_x.py:104-112 mean_of_dict = torch.mean of the stacked fp16 maxima)."""
        if self.count == 0:
            raise RuntimeError("calibration hook recorded no calls")
        if self.count > _MAX_CALLS:
            raise NotImplementedError(f"{self.count} calls: torch's cascade widens its levels past 2^16 rows")
        tot = self.acc[0].clone()
        for j in range(1, _LEVELS):
            tot += self.acc[j]
        return (tot / self.count).to(torch.float16)

    def clear(self):
        for a in self.acc:
            a.zero_()
        self.count = 0


class CalibrationSession:
    """apply_hook (calib_data.py:216-224) on every Linear of every smoothing block."""

    def __init__(self, blocks):
        self.blocks = blocks
        self.hooks = {}

    def attach(self):
        for bname, block in self.blocks.items():
            d = {}
            for name, sub in block.named_modules():
                if isinstance(sub, nn.Linear):
                    h = MeanMaxActivationHook(sub.in_features, sub.weight.device)
                    sub._qd_hook = h
                    d[name] = h
            self.hooks[bname] = d

    def detach(self):
        for block in self.blocks.values():
            for sub in block.modules():
                if hasattr(sub, "_qd_hook"):
                    del sub._qd_hook

    def clear(self):
        self.hooks = {}


def synthetic_calibration_set(n_samples=96, batch_size=8, seed=42, latent_shape=(4, 64, 64)):
    """[(prompts, latents)] batches with the reference's sizes and latent seed."""
    assert n_samples % batch_size == 0, "The batch_size, doesnt divide the dataset, choose an appropriate batch_size"
    gen = torch.manual_seed(seed)
    out = []
    for i in range(n_samples // batch_size):
        prompts = [f"calibration caption {i * batch_size + j}" for j in range(batch_size)]
        lat = torch.randn((batch_size, *latent_shape), generator=gen).to(torch.float16)
        out.append((prompts, lat))
    return out
