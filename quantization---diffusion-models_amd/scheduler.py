"""DDIM scheduler tables (diffusers DDIMScheduler, SD1.5 scheduler_config) for the device loop.

Only the per-step constants are computed here (host setup, as diffusers does); the step itself
is the fused ``qd_cfg_ddim_step`` kernel.  SD1.5 config: beta_start 0.00085, beta_end 0.012,
"scaled_linear", 1000 train steps, steps_offset 1, set_alpha_to_one False, "leading" spacing,
epsilon prediction, clip_sample False.  50 steps -> timesteps 981, 961, ..., 1.
"""
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class DDIMConfig:
    num_train_timesteps: int = 1000
    beta_start: float = 0.00085
    beta_end: float = 0.012
    beta_schedule: str = "scaled_linear"
    steps_offset: int = 1
    set_alpha_to_one: bool = False


def alphas_cumprod(cfg: DDIMConfig = DDIMConfig()):
    """float32 like diffusers (betas = linspace(sqrt(b0), sqrt(b1), T)**2 in float32)."""
    if cfg.beta_schedule == "scaled_linear":
        betas = torch.linspace(cfg.beta_start ** 0.5, cfg.beta_end ** 0.5, cfg.num_train_timesteps,
                               dtype=torch.float32) ** 2
    elif cfg.beta_schedule == "linear":
        betas = torch.linspace(cfg.beta_start, cfg.beta_end, cfg.num_train_timesteps, dtype=torch.float32)
    else:
        raise NotImplementedError(f"beta_schedule {cfg.beta_schedule}")
    return torch.cumprod(1.0 - betas, dim=0)


def ddim_tables(num_inference_steps, cfg: DDIMConfig = DDIMConfig()):
    """(timesteps int64 [S], alpha_t f32 [S], alpha_prev f32 [S]) for the 'leading' spacing."""
    ac = alphas_cumprod(cfg)
    final = torch.tensor(1.0) if cfg.set_alpha_to_one else ac[0]
    ratio = cfg.num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64) + cfg.steps_offset
    a_t = torch.stack([ac[int(t)] for t in ts])
    a_p = torch.stack([ac[int(t) - ratio] if int(t) - ratio >= 0 else final for t in ts])
    return torch.from_numpy(ts), a_t.float(), a_p.float()
