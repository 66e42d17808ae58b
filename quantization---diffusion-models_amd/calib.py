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


class MeanMaxActivationHook:
    def __init__(self, channels, device):
        self.sum = torch.zeros(channels, dtype=torch.float32, device=device)
        self.ws = torch.empty(channels, dtype=torch.float32, device=device)
        self.count = 0
        self.hook_handle = None

    def __call__(self, x2d):
        K.channel_absmax_accum(x2d, self.ws, self.sum)
        self.count += 1

    def mean(self):
        """mean over recorded calls, rounded to fp16 like torch.mean of a stacked fp16 list."""
        if self.count == 0:
            raise RuntimeError("calibration hook recorded no calls")
        return (self.sum / self.count).to(torch.float16)

    def clear(self):
        self.sum.zero_()
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
