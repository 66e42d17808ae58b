"""Pipeline container and local (offline) loading / saving of diffusers-format directories.

``QDiffPipeline`` stands in for the third-party ``diffusers.DiffusionPipeline`` the reference
wraps (models/base.py:199): it exposes ``components`` (the adapters bucket component names that
contain 'unet' / 'text_encoder' / 'vae' / 'transformer', StableDiffusion1_x.py:19-33),
``to(device)`` and ``save_pretrained``.  Weights load from a local diffusers directory
(``model_index.json`` + ``unet/config.json`` + ``unet/diffusion_pytorch_model.safetensors``) -
there is no network - or are synthesized (``synthetic:sd15`` / ``synthetic:sdxl`` /
``synthetic:tiny``) with SD shapes and N(0, 1/fan_in) values.
"""
import json
import os

import torch

from .scheduler import DDIMConfig
from .unet import SD15, SDXL, UNet2DConditionModel, UNetConfig, tiny_config

SYNTHETIC = {
    "synthetic:sd15": ("StableDiffusionPipeline", SD15),
    "synthetic:sdxl": ("StableDiffusionXLPipeline", SDXL),
    "synthetic:tiny": ("StableDiffusionPipeline", None),
}


class QDiffPipeline:
    def __init__(self, unet, class_name="StableDiffusionPipeline", scheduler_config=None, text_encoder=None,
                 vae=None, config=None):
        self.unet = unet
        self.text_encoder = text_encoder
        self.vae = vae
        self.scheduler_config = scheduler_config or DDIMConfig()
        self.class_name = class_name
        self.config = config or {"_class_name": class_name}
        self.device = next(unet.parameters()).device

    @property
    def components(self):
        return {"unet": self.unet, "text_encoder": self.text_encoder, "vae": self.vae,
                "scheduler": self.scheduler_config}

    def to(self, device):
        self.unet.to(device)
        self.device = torch.device(device)
        return self

    def save_pretrained(self, save_dir, safe_serialization=True):
        from safetensors.torch import save_file
        os.makedirs(os.path.join(save_dir, "unet"), exist_ok=True)
        with open(os.path.join(save_dir, "model_index.json"), "w") as f:
            json.dump({"_class_name": self.class_name, "unet": ["diffusers", "UNet2DConditionModel"],
                       "scheduler": ["diffusers", "DDIMScheduler"]}, f, indent=2)
        cfg = dict(vars(self.unet.config))
        cfg = {k: (list(v) if isinstance(v, tuple) else v) for k, v in cfg.items()}
        cfg["_class_name"] = "UNet2DConditionModel"
        with open(os.path.join(save_dir, "unet", "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        sd = {k: v.detach().to("cpu").contiguous() for k, v in self.unet.state_dict().items()}
        save_file(sd, os.path.join(save_dir, "unet", "diffusion_pytorch_model.safetensors"))


def load_config(model_path):
    if model_path in SYNTHETIC:
        return {"_class_name": SYNTHETIC[model_path][0]}
    p = os.path.join(model_path, "model_index.json")
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{model_path!r} is not a local diffusers directory (no model_index.json). There is no network "
            "access here: pass a local directory, or 'synthetic:sd15' / 'synthetic:sdxl' / 'synthetic:tiny'.")
    with open(p) as f:
        return json.load(f)


def load_pipeline(model_path, device="cuda", seed=0, dtype=torch.float16):
    cfg = load_config(model_path)
    cls = cfg["_class_name"]
    if model_path in SYNTHETIC:
        ucfg = SYNTHETIC[model_path][1] or tiny_config()
        unet = UNet2DConditionModel(ucfg).to(dtype)
        unet.init_synthetic(seed)
    else:
        with open(os.path.join(model_path, "unet", "config.json")) as f:
            ucfg = UNetConfig.from_diffusers(json.load(f))
        unet = UNet2DConditionModel(ucfg).to(dtype)
        wpath = os.path.join(model_path, "unet", "diffusion_pytorch_model.safetensors")
        from safetensors.torch import load_file
        sd = load_file(wpath)
        missing, unexpected = unet.load_state_dict({k: v.to(dtype) for k, v in sd.items()}, strict=False)
        if missing:
            raise KeyError(f"UNet weights missing keys (first 5): {missing[:5]}")
    unet.to(device)
    unet.eval()
    return QDiffPipeline(unet, cls, config=cfg)
