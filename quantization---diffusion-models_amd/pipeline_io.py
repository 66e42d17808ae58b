"""Pipeline container and local (offline) loading / saving of diffusers-format directories.

``QDiffPipeline`` stands in for the third-party ``diffusers.DiffusionPipeline`` the reference
wraps (models/base.py:199): it exposes ``components`` (the adapters bucket component names that
contain 'unet' / 'text_encoder' / 'vae' / 'transformer', StableDiffusion1_x.py:19-33,
StableDiffusion3_5.py:17-31), ``to(device)`` and ``save_pretrained``.  Weights load from a local
diffusers directory (``model_index.json`` + ``unet/`` or ``transformer/`` ``config.json`` +
``diffusion_pytorch_model.safetensors``) - there is no network - or are synthesized
(``synthetic:sd15`` / ``synthetic:sdxl`` / ``synthetic:tiny`` / ``synthetic:sdxl-tiny`` /
``synthetic:sd35`` / ``synthetic:sd35-medium`` / ``synthetic:sd35-tiny`` / ``synthetic:sd35m-tiny``) with the real shapes and N(0, 1/fan_in) values.
"""
import json
import os

import torch

from .mmdit import SD35_LARGE, SD35_MEDIUM, MMDiTConfig, SD3Transformer2DModel, tiny_mmdit_config
from .scheduler import (DDIMConfig, EulerDiscreteConfig, FlowMatchConfig, PNDMConfig, config_from_diffusers,
                        config_to_diffusers)
from .unet import SD15, SDXL, UNet2DConditionModel, UNetConfig, tiny_config, tiny_sdxl_config

SYNTHETIC = {
    "synthetic:sd15": ("StableDiffusionPipeline", SD15),
    "synthetic:sdxl": ("StableDiffusionXLPipeline", SDXL),
    "synthetic:tiny": ("StableDiffusionPipeline", None),
    "synthetic:sdxl-tiny": ("StableDiffusionXLPipeline", None),
    "synthetic:sd35": ("StableDiffusion3Pipeline", SD35_LARGE),
    "synthetic:sd35-tiny": ("StableDiffusion3Pipeline", None),
    "synthetic:sd35-medium": ("StableDiffusion3Pipeline", SD35_MEDIUM),
    # SD3.5-Medium-shaped tiny MMDiT-X: dual attention in blocks 0-1 of 3 (block 2 is context_pre_only)
    "synthetic:sd35m-tiny": ("StableDiffusion3Pipeline", tiny_mmdit_config(num_layers=3, dual_attention_layers=(0, 1))),
}
MMDIT_PIPELINES = ("StableDiffusion3Pipeline",)


class QDiffPipeline:
    def __init__(self, unet=None, class_name="StableDiffusionPipeline", scheduler_config=None, text_encoder=None,
                 vae=None, config=None, transformer=None):
        if (unet is None) == (transformer is None):
            raise ValueError("a pipeline holds exactly one denoiser: a unet or a transformer")
        self.unet = unet
        self.transformer = transformer
        self.text_encoder = text_encoder
        self.vae = vae
        if scheduler_config is None:
            scheduler_config = (FlowMatchConfig() if transformer is not None else
                                EulerDiscreteConfig() if class_name == "StableDiffusionXLPipeline" else DDIMConfig())
        self.scheduler_config = scheduler_config
        self.class_name = class_name
        self.config = config or {"_class_name": class_name}
        self.device = next(self.denoiser.parameters()).device

    @property
    def denoiser(self):
        return self.unet if self.unet is not None else self.transformer

    @property
    def denoiser_name(self):
        return "unet" if self.unet is not None else "transformer"

    @property
    def components(self):
        comps = {"text_encoder": self.text_encoder, "vae": self.vae, "scheduler": self.scheduler_config}
        comps[self.denoiser_name] = self.denoiser
        return comps

    def to(self, device):
        self.denoiser.to(device)
        self.device = torch.device(device)
        return self

    def save_pretrained(self, save_dir, safe_serialization=True):
        from safetensors.torch import save_file
        name = self.denoiser_name
        os.makedirs(os.path.join(save_dir, name), exist_ok=True)
        sched = config_to_diffusers(self.scheduler_config)
        if name == "unet":
            index = {"unet": ["diffusers", "UNet2DConditionModel"], "scheduler": ["diffusers", sched["_class_name"]]}
            cls = "UNet2DConditionModel"
        else:
            index = {"transformer": ["diffusers", "SD3Transformer2DModel"],
                     "scheduler": ["diffusers", sched["_class_name"]]}
            cls = "SD3Transformer2DModel"
        with open(os.path.join(save_dir, "model_index.json"), "w") as f:
            json.dump({"_class_name": self.class_name, **index}, f, indent=2)
        os.makedirs(os.path.join(save_dir, "scheduler"), exist_ok=True)
        with open(os.path.join(save_dir, "scheduler", "scheduler_config.json"), "w") as f:
            json.dump(sched, f, indent=2)
        cfg = dict(vars(self.denoiser.config))
        cfg = {k: (list(v) if isinstance(v, tuple) else v) for k, v in cfg.items()}
        cfg["_class_name"] = cls
        with open(os.path.join(save_dir, name, "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        sd = {k: v.detach().to("cpu").contiguous() for k, v in self.denoiser.state_dict().items()}
        save_file(sd, os.path.join(save_dir, name, "diffusion_pytorch_model.safetensors"))


def load_config(model_path):
    if model_path in SYNTHETIC:
        return {"_class_name": SYNTHETIC[model_path][0]}
    p = os.path.join(model_path, "model_index.json")
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{model_path!r} is not a local diffusers directory (no model_index.json). There is no network "
            "access here: pass a local directory, or one of " + ", ".join(repr(k) for k in SYNTHETIC) + ".")
    with open(p) as f:
        return json.load(f)


def _load_weights(module, path, dtype):
    from safetensors.torch import load_file
    sd = load_file(path)
    missing, unexpected = module.load_state_dict({k: v.to(dtype) for k, v in sd.items()}, strict=False)
    if missing:
        raise KeyError(f"weights missing keys (first 5): {missing[:5]}")


def load_scheduler_config(model_path, override=None):
    """The checkpoint's scheduler (scheduler/scheduler_config.json), as diffusers'
    DiffusionPipeline.from_pretrained instantiates it (the reference's generate() runs that
    scheduler, models/base.py:848); override: "ddim" / "pndm" / "euler" or a config object."""
    if override is not None and not isinstance(override, str):
        return override
    if isinstance(override, str):
        return {"ddim": DDIMConfig, "pndm": PNDMConfig, "euler": EulerDiscreteConfig,
                "flowmatch": FlowMatchConfig}[override.lower()]()
    if model_path in SYNTHETIC:
        return None  # synthetic checkpoints: the measurement protocol's DDIM / model defaults
    p = os.path.join(model_path, "scheduler", "scheduler_config.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return config_from_diffusers(json.load(f))


def load_pipeline(model_path, device="cuda", seed=0, dtype=torch.float16, scheduler=None):
    cfg = load_config(model_path)
    cls = cfg["_class_name"]
    mmdit = cls in MMDIT_PIPELINES
    sched_cfg = load_scheduler_config(model_path, scheduler)
    if model_path in SYNTHETIC:
        mcfg = SYNTHETIC[model_path][1] or (tiny_mmdit_config() if mmdit else
                                            tiny_sdxl_config() if cls == "StableDiffusionXLPipeline" else tiny_config())
        if mmdit:
            # built and drawn on the target device (a full SD3.5-Large is 8 B parameters)
            with torch.device(device):
                net = SD3Transformer2DModel(mcfg).to(dtype)
            big = not model_path.endswith("-tiny") and torch.device(device).type == "cuda"
            net.init_synthetic(seed, rng_device=device if big else "cpu")
        else:
            net = UNet2DConditionModel(mcfg).to(dtype)
            net.init_synthetic(seed)
    else:
        sub = "transformer" if mmdit else "unet"
        with open(os.path.join(model_path, sub, "config.json")) as f:
            c = json.load(f)
        if mmdit:
            net = SD3Transformer2DModel(MMDiTConfig.from_diffusers(c)).to(dtype)
        else:
            net = UNet2DConditionModel(UNetConfig.from_diffusers(c)).to(dtype)
        _load_weights(net, os.path.join(model_path, sub, "diffusion_pytorch_model.safetensors"), dtype)
    net.to(device)
    net.eval()
    if mmdit:
        return QDiffPipeline(transformer=net, class_name=cls, config=cfg, scheduler_config=sched_cfg)
    return QDiffPipeline(net, cls, config=cfg, scheduler_config=sched_cfg)
