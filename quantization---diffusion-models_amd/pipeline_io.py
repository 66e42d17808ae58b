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


AUX_COMPONENTS = ("text_encoder", "text_encoder_2", "tokenizer", "tokenizer_2", "vae")


class QDiffPipeline:
    """Denoiser + scheduler config + the aux components (text encoder(s), tokenizers, VAE).
    `lazy` maps aux component names to zero-argument factories: synthetic checkpoints and local
    directories build their text encoders / VAE only when a prompt string must be encoded or
    latents decoded (the denoising loop never needs them)."""

    def __init__(self, unet=None, class_name="StableDiffusionPipeline", scheduler_config=None, text_encoder=None,
                 vae=None, config=None, transformer=None, text_encoder_2=None, tokenizer=None, tokenizer_2=None,
                 lazy=None):
        if (unet is None) == (transformer is None):
            raise ValueError("a pipeline holds exactly one denoiser: a unet or a transformer")
        self.unet = unet
        self.transformer = transformer
        self._lazy = dict(lazy or {})
        given = dict(text_encoder=text_encoder, text_encoder_2=text_encoder_2, tokenizer=tokenizer,
                     tokenizer_2=tokenizer_2, vae=vae)
        for name, obj in given.items():
            if obj is not None or name not in self._lazy:
                self._lazy.pop(name, None)
                setattr(self, name, obj)
        if scheduler_config is None:
            scheduler_config = (FlowMatchConfig() if transformer is not None else
                                EulerDiscreteConfig() if class_name == "StableDiffusionXLPipeline" else DDIMConfig())
        self.scheduler_config = scheduler_config
        self.class_name = class_name
        self.config = config or {"_class_name": class_name}
        self.device = next(self.denoiser.parameters()).device

    def __getattr__(self, name):
        lazy = self.__dict__.get("_lazy")
        if lazy is not None and name in lazy:
            obj = lazy.pop(name)(self)
            setattr(self, name, obj)
            return obj
        raise AttributeError(name)

    @property
    def denoiser(self):
        return self.unet if self.unet is not None else self.transformer

    @property
    def denoiser_name(self):
        return "unet" if self.unet is not None else "transformer"

    def component_names(self):
        """Names of the model components present (built or buildable), denoiser first."""
        names = [self.denoiser_name]
        for n in ("text_encoder", "text_encoder_2", "vae"):
            if n in self._lazy or self.__dict__.get(n) is not None:
                names.append(n)
        return names

    @property
    def components(self):
        """diffusers' DiffusionPipeline.components: every model slot (None when absent; lazy ones
        are built by this access) and the scheduler."""
        comps = {self.denoiser_name: self.denoiser, "text_encoder": None, "vae": None}
        for n in self.component_names()[1:]:
            comps[n] = getattr(self, n)
        comps["scheduler"] = self.scheduler_config
        return comps

    def built_aux(self):
        return {n: self.__dict__[n] for n in ("text_encoder", "text_encoder_2", "vae")
                if self.__dict__.get(n) is not None}

    def to(self, device):
        self.denoiser.to(device)
        for m in self.built_aux().values():
            m.to(device)
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
        for aux, m in self.built_aux().items():   # text encoders / VAE that were built (or loaded)
            d = os.path.join(save_dir, aux)
            os.makedirs(d, exist_ok=True)
            if aux.startswith("text_encoder"):
                arch = "CLIPTextModelWithProjection" if m.config.projection_dim else "CLIPTextModel"
                c, fname, index[aux] = dict(m.config.to_transformers(), architectures=[arch]), "model.safetensors", \
                    ["transformers", arch]
            else:
                c, fname, index[aux] = m.config.to_diffusers(), "diffusion_pytorch_model.safetensors", \
                    ["diffusers", "AutoencoderKL"]
            with open(os.path.join(d, "config.json"), "w") as f:
                json.dump(c, f, indent=2)
            save_file({k: v.detach().to("cpu").contiguous() for k, v in m.state_dict().items()},
                      os.path.join(d, fname))
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


def _load_weights(module, path, dtype, rename=None):
    from safetensors.torch import load_file
    sd = load_file(path)
    if rename is not None:
        sd = {rename(k): v for k, v in sd.items()}
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


# ------------------------------------------------------------------ text encoders / VAE
def _te_factory(cfg, seed=None, path=None):
    def build(pipe):
        from .clip import CLIPTextModel
        m = CLIPTextModel(cfg).half()
        if path is None:
            m.init_synthetic(seed)
        else:
            _load_weights(m, _first(path, ("model.safetensors", "model.fp16.safetensors")), torch.float16,
                          rename=_clip_keys)
        return m.to(pipe.device).eval()
    return build


def _vae_factory(cfg, seed=None, path=None):
    def build(pipe):
        from .vae import AutoencoderKL
        m = AutoencoderKL(cfg).half()
        if path is None:
            m.init_synthetic(seed)
        else:
            _load_weights(m, _first(path, ("diffusion_pytorch_model.safetensors",
                                           "diffusion_pytorch_model.fp16.safetensors")), torch.float16,
                          rename=_vae_keys)
        return m.to(pipe.device).eval()
    return build


def _first(d, names):
    for n in names:
        if os.path.exists(os.path.join(d, n)):
            return os.path.join(d, n)
    raise FileNotFoundError(f"no weights file ({', '.join(names)}) in {d}")


def _clip_keys(k):
    """transformers >= 5 may save CLIPTextModel without the text_model. prefix."""
    if k.startswith(("embeddings.", "encoder.", "final_layer_norm.")):
        return "text_model." + k
    return k


_VAE_LEGACY = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}


def _vae_keys(k):
    """diffusers' legacy VAE attention names (query / key / value / proj_attn)."""
    for a, b in _VAE_LEGACY.items():
        k = k.replace(a, b)
    return k


def _synthetic_aux(cls, mcfg, tiny, seed):
    """{component: factory(pipeline)} of a synthetic checkpoint's text encoder(s), tokenizers and
    VAE: the real architectures (CLIP ViT-L/14, OpenCLIP bigG, AutoencoderKL) for full-size
    models, small ones sized to the denoiser's conditioning widths for the tiny test models."""
    from .clip import CLIP_G, CLIP_L, CLIP_L_PROJ, EOS, HashTokenizer, tiny_clip_config
    from .vae import SD3_VAE, SD_VAE, SDXL_VAE, tiny_vae_config
    tok1, tok2 = (lambda p: HashTokenizer(pad_id=EOS)), (lambda p: HashTokenizer(pad_id=0))
    if cls == "StableDiffusionPipeline":
        te = tiny_clip_config(hidden=mcfg.cross_attention_dim) if tiny else CLIP_L
        return {"text_encoder": _te_factory(te, seed + 1), "tokenizer": tok1,
                "vae": _vae_factory(tiny_vae_config() if tiny else SD_VAE, seed + 3)}
    if cls == "StableDiffusionXLPipeline":
        if tiny:
            cross = mcfg.cross_attention_dim
            pooled = mcfg.projection_class_embeddings_input_dim - 6 * mcfg.addition_time_embed_dim
            te1 = tiny_clip_config(hidden=cross // 2)
            te2 = tiny_clip_config(hidden=cross - cross // 2, projection_dim=pooled, act="gelu")
        else:
            te1, te2 = CLIP_L, CLIP_G
        return {"text_encoder": _te_factory(te1, seed + 1), "text_encoder_2": _te_factory(te2, seed + 2),
                "tokenizer": tok1, "tokenizer_2": tok2,
                "vae": _vae_factory(tiny_vae_config() if tiny else SDXL_VAE, seed + 3)}
    if tiny:
        pd = mcfg.pooled_projection_dim
        te1 = tiny_clip_config(hidden=pd // 2, projection_dim=pd // 2)
        te2 = tiny_clip_config(hidden=pd - pd // 2, projection_dim=pd - pd // 2, act="gelu")
    else:
        te1, te2 = CLIP_L_PROJ, CLIP_G
    return {"text_encoder": _te_factory(te1, seed + 1), "text_encoder_2": _te_factory(te2, seed + 2),
            "tokenizer": tok1, "tokenizer_2": tok2,
            "vae": _vae_factory(tiny_vae_config(16) if tiny else SD3_VAE, seed + 3)}


def _local_aux(model_path):
    """{component: factory(pipeline)} for the text encoder / tokenizer / VAE sub-directories a
    local diffusers checkpoint holds (text_encoder_3 / T5 is not supported: SD3 prompts encode
    with the two CLIP encoders and zero T5 features, as diffusers does without it)."""
    from .clip import EOS, CLIPTextConfig, load_tokenizer
    from .vae import VAEConfig
    out = {}
    for name in ("text_encoder", "text_encoder_2"):
        d = os.path.join(model_path, name)
        if os.path.exists(os.path.join(d, "config.json")):
            with open(os.path.join(d, "config.json")) as f:
                c = json.load(f)
            proj = any("WithProjection" in a for a in c.get("architectures", []))
            out[name] = _te_factory(CLIPTextConfig.from_transformers(c, with_projection=proj), path=d)
    for name, pad in (("tokenizer", EOS), ("tokenizer_2", 0)):
        d = os.path.join(model_path, name)
        if os.path.isdir(d):
            out[name] = (lambda p, d=d, pad=pad: load_tokenizer(d, pad_id=pad))
    d = os.path.join(model_path, "vae")
    if os.path.exists(os.path.join(d, "config.json")):
        with open(os.path.join(d, "config.json")) as f:
            out["vae"] = _vae_factory(VAEConfig.from_diffusers(json.load(f)), path=d)
    return out


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
        lazy = _synthetic_aux(cls, mcfg, SYNTHETIC[model_path][1] is None or model_path.endswith("-tiny"), seed)
    else:
        sub = "transformer" if mmdit else "unet"
        with open(os.path.join(model_path, sub, "config.json")) as f:
            c = json.load(f)
        if mmdit:
            net = SD3Transformer2DModel(MMDiTConfig.from_diffusers(c)).to(dtype)
        else:
            net = UNet2DConditionModel(UNetConfig.from_diffusers(c)).to(dtype)
        _load_weights(net, os.path.join(model_path, sub, "diffusion_pytorch_model.safetensors"), dtype)
        lazy = _local_aux(model_path)
    net.to(device)
    net.eval()
    if mmdit:
        return QDiffPipeline(transformer=net, class_name=cls, config=cfg, scheduler_config=sched_cfg, lazy=lazy)
    return QDiffPipeline(net, cls, config=cfg, scheduler_config=sched_cfg, lazy=lazy)
