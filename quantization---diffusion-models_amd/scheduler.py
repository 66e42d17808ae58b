"""Scheduler tables for the device loops: DDIM (diffusers DDIMScheduler, SD1.5
scheduler_config), Euler discrete (EulerDiscreteScheduler, the SDXL base scheduler_config) and
flow-match Euler (FlowMatchEulerDiscreteScheduler, SD3 / SD3.5).

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


@dataclass
class FlowMatchConfig:
    """FlowMatchEulerDiscreteScheduler config of the SD3 / SD3.5 pipelines."""
    num_train_timesteps: int = 1000
    shift: float = 3.0


def flowmatch_tables(num_inference_steps, cfg: FlowMatchConfig = FlowMatchConfig()):
    """(timesteps f32 [S], sigmas f32 [S + 1]) of FlowMatchEulerDiscreteScheduler.set_timesteps
    (static shift): the training sigmas t/T (float32) are shifted s*x / (1 + (s-1)*x), their
    ends span a float64 linspace of S timesteps, which are shifted again; sigmas end with 0."""
    n_t = cfg.num_train_timesteps
    train = torch.from_numpy(np.linspace(1, n_t, n_t, dtype=np.float32)[::-1].copy()) / n_t
    train = cfg.shift * train / (1 + (cfg.shift - 1) * train)
    hi, lo = train[0].item() * n_t, train[-1].item() * n_t
    sig = np.linspace(hi, lo, num_inference_steps) / n_t
    sig = torch.from_numpy(cfg.shift * sig / (1 + (cfg.shift - 1) * sig)).to(torch.float32)
    return sig * n_t, torch.cat([sig, torch.zeros(1)])


def ddim_tables(num_inference_steps, cfg: DDIMConfig = DDIMConfig()):
    """(timesteps int64 [S], alpha_t f32 [S], alpha_prev f32 [S]) for the 'leading' spacing."""
    ac = alphas_cumprod(cfg)
    final = torch.tensor(1.0) if cfg.set_alpha_to_one else ac[0]
    ratio = cfg.num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64) + cfg.steps_offset
    a_t = torch.stack([ac[int(t)] for t in ts])
    a_p = torch.stack([ac[int(t) - ratio] if int(t) - ratio >= 0 else final for t in ts])
    return torch.from_numpy(ts), a_t.float(), a_p.float()


@dataclass
class PNDMConfig(DDIMConfig):
    """PNDMScheduler of the SD1.5 checkpoints (scheduler/scheduler_config.json: skip_prk_steps
    true, steps_offset 1, set_alpha_to_one false, the SD1.5 betas): the scheduler the reference's
    generate() runs through the pipeline (models/base.py:848)."""
    skip_prk_steps: bool = True


def pndm_tables(num_inference_steps, cfg: PNDMConfig = PNDMConfig()):
    """(timesteps int64 [S + 1], alpha_t f32 [S + 1], alpha_prev f32 [S + 1]) of
    PNDMScheduler.set_timesteps + step_plms (skip_prk_steps): the PLMS timesteps repeat the
    second one ([981, 961, 961, 941, ..., 1] for 50 steps, S + 1 UNet evaluations); step 1
    re-evaluates step 0's interval (alphas of t + ratio -> t); prev_t < 0 -> final_alpha_cumprod."""
    if not cfg.skip_prk_steps:
        raise NotImplementedError("PNDM Runge-Kutta (prk) warm-up steps: the SD pipelines set skip_prk_steps")
    ac = alphas_cumprod(cfg)
    final = torch.tensor(1.0) if cfg.set_alpha_to_one else ac[0]
    ratio = cfg.num_train_timesteps // num_inference_steps
    t = (np.arange(0, num_inference_steps) * ratio).round().astype(np.int64) + cfg.steps_offset
    ts = np.concatenate([t[:-1], t[-2:-1], t[-1:]])[::-1].copy()
    a_t, a_p = [], []
    for i, ti in enumerate(ts):
        cur, prev = (int(ti) + ratio, int(ti)) if i == 1 else (int(ti), int(ti) - ratio)
        a_t.append(ac[cur])
        a_p.append(ac[prev] if prev >= 0 else final)
    return torch.from_numpy(ts), torch.stack(a_t).float(), torch.stack(a_p).float()


_SPACING_DEFAULT = {"EulerDiscreteScheduler": "linspace"}


def config_from_diffusers(d):
    """A scheduler config object from a diffusers scheduler_config.json dict (the local
    checkpoint's own scheduler, as DiffusionPipeline.from_pretrained would build it)."""
    name = d.get("_class_name", "DDIMScheduler")
    if name == "FlowMatchEulerDiscreteScheduler":
        return FlowMatchConfig(num_train_timesteps=d.get("num_train_timesteps", 1000), shift=d.get("shift", 3.0))
    cls = {"DDIMScheduler": DDIMConfig, "PNDMScheduler": PNDMConfig,
           "EulerDiscreteScheduler": EulerDiscreteConfig}.get(name)
    if cls is None:
        raise NotImplementedError(f"scheduler {name} has no device step kernel in this build")
    kw = {k: d[k] for k in ("num_train_timesteps", "beta_start", "beta_end", "beta_schedule", "steps_offset",
                            "set_alpha_to_one") if k in d}
    if cls is PNDMConfig and "skip_prk_steps" in d:
        kw["skip_prk_steps"] = d["skip_prk_steps"]
    if d.get("prediction_type", "epsilon") != "epsilon":
        raise NotImplementedError(f"prediction_type {d['prediction_type']}: the SD pipelines use epsilon")
    # the device step kernels implement "leading" spacing without sample clipping / dynamic
    # thresholding: a config asking for anything else would silently run another schedule than
    # DiffusionPipeline.from_pretrained builds from the same file
    # (a missing key means the class's own default: diffusers' EulerDiscreteScheduler defaults to
    # "linspace", DDIM and PNDM to "leading")
    spacing = d.get("timestep_spacing", _SPACING_DEFAULT.get(name, "leading"))
    if spacing != "leading":
        raise NotImplementedError(f"{name} timestep_spacing {spacing!r} (only 'leading')")
    if d.get("thresholding", False):
        raise NotImplementedError(f"{name} thresholding=True (dynamic thresholding) has no device kernel")
    if name == "DDIMScheduler" and d.get("clip_sample", True):  # diffusers' DDIM default is True
        raise NotImplementedError("DDIMScheduler clip_sample=True has no device kernel (SD checkpoints set False)")
    return cls(**kw)


def config_to_diffusers(cfg):
    """scheduler_config.json dict of a scheduler config object (save_pretrained)."""
    if isinstance(cfg, FlowMatchConfig):
        return {"_class_name": "FlowMatchEulerDiscreteScheduler", "num_train_timesteps": cfg.num_train_timesteps,
                "shift": cfg.shift}
    name = {PNDMConfig: "PNDMScheduler", EulerDiscreteConfig: "EulerDiscreteScheduler"}.get(type(cfg), "DDIMScheduler")
    d = {"_class_name": name, "num_train_timesteps": cfg.num_train_timesteps, "beta_start": cfg.beta_start,
         "beta_end": cfg.beta_end, "beta_schedule": cfg.beta_schedule, "steps_offset": cfg.steps_offset,
         "set_alpha_to_one": cfg.set_alpha_to_one, "prediction_type": "epsilon"}
    if isinstance(cfg, PNDMConfig):
        d["skip_prk_steps"] = cfg.skip_prk_steps
    d["timestep_spacing"] = "leading"
    if name == "DDIMScheduler":
        d["clip_sample"] = False
    return d


@dataclass
class EulerDiscreteConfig(DDIMConfig):
    """EulerDiscreteScheduler of the SDXL base pipeline: the SD1.5 beta schedule, "leading"
    timestep spacing with steps_offset 1, epsilon prediction, linear sigma interpolation."""


def euler_discrete_tables(num_inference_steps, cfg: EulerDiscreteConfig = EulerDiscreteConfig()):
    """(timesteps f32 [S], sigmas f32 [S + 1], dscale f32 [S + 1], init_noise_sigma) of
    EulerDiscreteScheduler.set_timesteps: sigma(t) = sqrt((1 - acp) / acp) at the leading-spaced
    timesteps (np.interp at integer t), a trailing 0; dscale = (sigma ** 2 + 1) ** 0.5 is
    scale_model_input's divisor; init_noise_sigma = (max sigma ** 2 + 1) ** 0.5 ("leading")."""
    ac = alphas_cumprod(cfg)
    ratio = cfg.num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.float32)
    ts += cfg.steps_offset
    sig_all = np.asarray((((1 - ac) / ac) ** 0.5).numpy() if torch.is_tensor(ac) else ((1 - ac) / ac) ** 0.5)
    sig = np.interp(ts, np.arange(0, len(sig_all)), sig_all)
    sigmas = torch.from_numpy(np.concatenate([sig, [0.0]]).astype(np.float32))
    dscale = (sigmas ** 2 + 1) ** 0.5
    init = (sigmas.max() ** 2 + 1) ** 0.5
    return torch.from_numpy(ts), sigmas, dscale, init
