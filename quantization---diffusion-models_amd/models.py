"""Diffusion adapters: StableDiffusion1_x, StableDiffusionXL, StableDiffusion3_5 and the AWQ
facade (models/StableDiffusion1_x.py, StableDiffusionXL.py, StableDiffusion3_5.py; README's
``AWQ.from_pretrained`` dispatching on model_index.json ``_class_name``).

Component discovery, layer lists and the SmoothQuant groups follow the reference adapters:
  set_quantizable_components   StableDiffusion1_x.py:19-33
  get_model_layers_unet        :39-47  (top-level (name, child) of each unet)
  get_model_layers_te / _vae   :49-67  (vae: decoder children only)
  get_smoothing_blocks         :96-102 (every BasicTransformerBlock)
  mean_of_dict                 :104-112
  get_layers_for_scaling_unet  :115-150 (norm1 -> attn1.to_q/k/v, norm3 -> ff.net.0.proj;
                                         activation = mean of attn1.to_q's / ff.net.0.proj's hook)
"""
import torch

from .base import QUANTISABLE_COMPONENTS, BaseAWQForDiffusion
from .calib import synthetic_calibration_set
from .clip import encode_sd3, encode_sdxl
from .pipeline import EulerDiscreteDenoiseLoop, FlowMatchDenoiseLoop, synthetic_text_embeddings
from .pipeline_io import load_config
from .unet import BasicTransformerBlock


class _DiffusionAdapter(BaseAWQForDiffusion):
    has_unet = True
    has_transformer = False

    def __init__(self, pipeline, model_type, is_quantized, config, quant_config, refiner_path=None,
                 access_token=None):
        super().__init__(pipeline, model_type, is_quantized, config, quant_config)
        self.quantizable_components = {"unet": [], "text_encoder": [], "vae": [], "transformer": []}
        self.quantized_components = []
        self.refiner_pipeline = None
        self.set_quantizable_components()

    def set_quantizable_components(self):
        for component in self.pipeline.component_names():   # aux components stay unbuilt until used
            for key in QUANTISABLE_COMPONENTS:
                if key in component:
                    self.quantizable_components[key].append(component)
                    break

    def _layers(self, key, sub=None):
        out = []
        for comp in self.quantizable_components[key]:
            mod = getattr(self.pipeline, comp)
            if sub is not None:
                mod = getattr(mod, sub)
            out.append([(n, m) for n, m in mod.named_children()])
        return out

    def get_model_layers_unet(self):
        if not self.has_unet:
            raise Exception("NO UNET IN THIS MODEL")
        return self._layers("unet")

    def get_model_layers_te(self):
        return self._layers("text_encoder")

    def get_model_layers_vae(self):
        return self._layers("vae", "decoder")

    def get_model_layers_transformers(self):
        if not self.has_transformer:
            raise Exception(f"There is no transformer in this model, {type(self).__name__}")
        return self._layers("transformer")

    def get_root(self, component, idx):
        return getattr(self.pipeline, self.quantizable_components[component][idx])

    def get_components(self):
        return self.quantizable_components

    def get_unet(self):
        return self.pipeline.unet

    def get_pipeline(self):
        return self.pipeline

    def set_quantized_components(self, component):
        self.quantized_components.append(component)

    def get_debugModuleNames(self, *a, **k):
        return []

    def get_scalingStates(self, *a, **k):
        return []

    def get_projectionNames(self, *a, **k):
        return []

    # ---------------------------------------------------------------- SmoothQuant hooks
    def get_smoothing_blocks(self):
        return {name: m for name, m in self.pipeline.unet.named_modules() if isinstance(m, BasicTransformerBlock)}

    @staticmethod
    def mean_of_dict(hook):
        return hook.mean()

    def get_layers_for_scaling_unet(self, module, hooks):
        return [
            dict(prev_op=module.norm1, layers=[module.attn1.to_q, module.attn1.to_k, module.attn1.to_v],
                 activations_max=[self.mean_of_dict(hooks["attn1.to_q"]), self.mean_of_dict(hooks["attn1.to_k"]),
                                  self.mean_of_dict(hooks["attn1.to_v"])]),
            dict(prev_op=module.norm3, layers=[module.ff.net[0].proj],
                 activations_max=[self.mean_of_dict(hooks["ff.net.0.proj"])]),
        ]

    @torch.no_grad()
    def run_sq_calibration(self, n_samples=96, batch_size=8, seed=42, num_inference_steps=50, guidance_scale=7.5,
                           height=None, width=None):
        """run_calibration (calib_data.py:227-245) on device, eager (hooks fire per call)."""
        cfg = self.pipeline.unet.config
        hh = height or cfg.sample_size * 8
        ww = width or cfg.sample_size * 8
        samples = synthetic_calibration_set(n_samples, batch_size, seed, (cfg.in_channels, hh // 8, ww // 8))
        for prompts, lat in samples:
            self.generate(prompt=prompts, height=hh, width=ww, num_inference_steps=num_inference_steps,
                          guidance_scale=guidance_scale, lat=lat, output_type="latent", use_graph=False)
        self._loops = {}


class StableDiffusion1_x(_DiffusionAdapter):
    def __init__(self, pipeline, model_type, is_quantized, config, quant_config, access_token=None,
                 refiner_path=None):
        if refiner_path is not None:
            raise Exception("StableDiffusion1.5 has no refiner model, if there is its not supported")
        super().__init__(pipeline, model_type, is_quantized, config, quant_config)

    def checkQuantStatus(self, quantUnet=True, quantTextEncoder=False, quantVAE=False, quantTransformer=True):
        if quantTransformer:
            raise Exception("There is no Transformer in this Diffusion Model")


class StableDiffusionXL(_DiffusionAdapter):
    """SDXL adapter (models/StableDiffusionXL.py); generate() drives diffusers'
    StableDiffusionXLPipeline loop - EulerDiscreteScheduler, guidance 5.0, the "text_time"
    additional conditioning (pooled text embeddings + time_ids) - on device."""

    def checkQuantStatus(self, quantUnet=True, quantTextEncoder=False, quantVAE=False, quantTransformer=True):
        if quantTransformer:
            raise Exception("There is no Transformer in this Diffusion Model")

    def get_quantized_components(self):
        return self.quantizable_components

    def _xl_conditioning(self, prompt, negative_prompt, prompt_embeds, negative_prompt_embeds,
                         pooled_prompt_embeds, negative_pooled_prompt_embeds, height, width, original_size,
                         crops_coords_top_left, target_size):
        cfg = self.pipeline.unet.config
        dev = self.pipeline.device
        pooled_dim = cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim
        if prompt_embeds is None and self._has_text_encoder():
            ctx, text = encode_sdxl(self.pipeline, prompt, negative_prompt)
            b = ctx.shape[0] // 2
        else:
            if prompt_embeds is not None and negative_prompt_embeds is None and negative_prompt is None:
                # force_zeros_for_empty_prompt (the SDXL base config): zero negative conditioning
                negative_prompt_embeds = torch.zeros_like(prompt_embeds)
                if negative_pooled_prompt_embeds is None and pooled_prompt_embeds is not None:
                    negative_pooled_prompt_embeds = torch.zeros_like(pooled_prompt_embeds)
            ctx = self._text_context(prompt, negative_prompt, prompt_embeds, negative_prompt_embeds)
            b = ctx.shape[0] // 2
            if pooled_prompt_embeds is None:
                prompts = [prompt] * b if isinstance(prompt, str) else list(prompt or [f"prompt{i}" for i in range(b)])
                pooled_prompt_embeds = synthetic_text_embeddings([f"{p}\x00pooled" for p in prompts], seq_len=1,
                                                                 dim=pooled_dim, device=dev)[:, 0]
            if negative_pooled_prompt_embeds is None:
                neg = negative_prompt if negative_prompt is not None else ""
                negs = [neg] * b if isinstance(neg, str) else list(neg)
                negative_pooled_prompt_embeds = synthetic_text_embeddings([f"{p}\x00pooled" for p in negs], seq_len=1,
                                                                          dim=pooled_dim, device=dev)[:, 0]
            text = torch.cat([negative_pooled_prompt_embeds.to(dev), pooled_prompt_embeds.to(dev)])
        text = text.to(torch.float16)
        # StableDiffusionXLPipeline._get_add_time_ids: original_size + crops_coords_top_left + target_size
        ids = list(original_size or (height, width)) + list(crops_coords_top_left) + list(target_size or (height, width))
        time_ids = torch.tensor([ids] * (2 * b), dtype=torch.float32)
        return ctx, text.contiguous(), time_ids

    def get_loop(self, batch, height, width, steps, guidance, use_graph=True):
        key = (batch, height, width, steps, float(guidance), use_graph)
        if key not in self._loops:
            self._loops[key] = EulerDiscreteDenoiseLoop(self.pipeline.unet, batch, height, width, steps, guidance,
                                                        device=self.pipeline.device, use_graph=use_graph,
                                                        sched_cfg=self.pipeline.scheduler_config)
        return self._loops[key]

    @torch.no_grad()
    def generate(self, prompt=None, height=1024, width=1024, num_inference_steps=50, guidance_scale=5.0,
                 negative_prompt=None, num_images_per_prompt=1, generator=None, device="cpu", lat=None,
                 output_type=None, prompt_embeds=None, negative_prompt_embeds=None, pooled_prompt_embeds=None,
                 negative_pooled_prompt_embeds=None, original_size=None, crops_coords_top_left=(0, 0),
                 target_size=None, use_graph=True, **kwargs):
        """base.py:828-850 for StableDiffusionXLPipeline (its default guidance 5.0; the reference
        passes 50 steps) -> the device Euler-discrete loop and the VAE decode (see base generate)."""
        if self.pipeline is None:
            raise RuntimeError("The diffusion pipeline is not loaded. Please use `from_pretrained` or `from_quantized` first.")
        ctx, text, time_ids = self._xl_conditioning(prompt, negative_prompt, prompt_embeds, negative_prompt_embeds,
                                                    pooled_prompt_embeds, negative_pooled_prompt_embeds, height, width,
                                                    original_size, crops_coords_top_left, target_size)
        if num_images_per_prompt > 1:
            b0, r = ctx.shape[0] // 2, num_images_per_prompt
            rep = lambda t: torch.cat([t[:b0].repeat_interleave(r, 0), t[b0:].repeat_interleave(r, 0)])
            ctx, text, time_ids = rep(ctx), rep(text), rep(time_ids)
        b = ctx.shape[0] // 2
        cin = self.pipeline.unet.config.in_channels
        if lat is None:
            lat = torch.randn((b, cin, height // 8, width // 8), generator=generator, dtype=torch.float32).to(torch.float16)
        loop = self.get_loop(b, height, width, num_inference_steps, guidance_scale, use_graph)
        return self._decode(loop.run(lat.to(self.pipeline.device), ctx, text, time_ids), output_type)


class StableDiffusion3_5(_DiffusionAdapter):
    """SD3 / SD3.5 MMDiT adapter (models/StableDiffusion3_5.py): the transformer component is
    quantized with quantTransformer=True (quantizer.py:1063-1064) and generate() drives the
    flow-match denoising loop of diffusers' StableDiffusion3Pipeline on device."""
    has_unet = False
    has_transformer = True

    def __init__(self, pipeline, model_type, is_quantized, config, quant_config, refiner_path=None,
                 access_token=None):
        if refiner_path is not None:
            raise Exception("StableDiffusion3.5 has no refiner model, if there is its not supported")
        super().__init__(pipeline, model_type, is_quantized, config, quant_config)

    def checkQuantStatus(self, quantUnet=True, quantTextEncoder=False, quantVAE=False, quantTransformer=True):
        if quantUnet:
            raise Exception("There is no UNET in StableDiffusion3_5")

    def get_transformer(self):
        return self.pipeline.transformer

    def get_unet(self):
        raise Exception("NO UNET IN THIS MODEL")

    def get_smoothing_blocks(self):
        raise NotImplementedError("SmoothQuant (quantType='sq') has no SD3.5 block mapping in the reference "
                                  "(StableDiffusion3_5.py defines no get_layers_for_scaling_unet)")

    def _text_context(self, prompt, negative_prompt, prompt_embeds, negative_prompt_embeds,
                      pooled_prompt_embeds=None, negative_pooled_prompt_embeds=None, seq_len=333):
        """[neg; pos] sequence embeddings [2B, Sc, joint_attention_dim] and pooled CLIP embeddings
        [2B, pooled_projection_dim]: the two CLIP encoders (zero T5 features) when the pipeline has
        them (clip.encode_sd3), else deterministic synthetic stand-ins."""
        cfg = self.pipeline.transformer.config
        dev = self.pipeline.device
        if prompt_embeds is None and self._has_text_encoder():
            return encode_sd3(self.pipeline, prompt, negative_prompt, joint_dim=cfg.joint_attention_dim)
        if prompt_embeds is None:
            prompts = [prompt] if isinstance(prompt, str) else list(prompt)
            prompt_embeds = synthetic_text_embeddings(prompts, seq_len=seq_len, dim=cfg.joint_attention_dim,
                                                      device=dev)
        else:
            prompts = None
        b = prompt_embeds.shape[0]
        if pooled_prompt_embeds is None:
            names = [f"{p}\x00pooled" for p in prompts] if prompts else [f"pooled{i}" for i in range(b)]
            pooled_prompt_embeds = synthetic_text_embeddings(names, seq_len=1, dim=cfg.pooled_projection_dim,
                                                             device=dev)[:, 0]
        neg = negative_prompt if negative_prompt is not None else ""
        negs = [neg] * b if isinstance(neg, str) else list(neg)
        if negative_prompt_embeds is None:
            negative_prompt_embeds = synthetic_text_embeddings(negs, seq_len=prompt_embeds.shape[1],
                                                               dim=cfg.joint_attention_dim, device=dev)
        if negative_pooled_prompt_embeds is None:
            negative_pooled_prompt_embeds = synthetic_text_embeddings([f"{p}\x00pooled" for p in negs], seq_len=1,
                                                                      dim=cfg.pooled_projection_dim, device=dev)[:, 0]
        ctx = torch.cat([negative_prompt_embeds.to(dev), prompt_embeds.to(dev)]).to(torch.float16).contiguous()
        pooled = torch.cat([negative_pooled_prompt_embeds.to(dev), pooled_prompt_embeds.to(dev)])
        return ctx, pooled.to(torch.float16).contiguous()

    def get_loop(self, batch, height, width, steps, guidance, use_graph=True, ctx_len=333):
        key = (batch, height, width, steps, float(guidance), use_graph, ctx_len)
        if key not in self._loops:
            self._loops[key] = FlowMatchDenoiseLoop(self.pipeline.transformer, batch, height, width, steps, guidance,
                                                    device=self.pipeline.device, use_graph=use_graph,
                                                    sched_cfg=self.pipeline.scheduler_config, ctx_len=ctx_len)
        return self._loops[key]

    @torch.no_grad()
    def generate(self, prompt=None, height=1024, width=1024, num_inference_steps=50, guidance_scale=7.0,
                 negative_prompt=None, num_images_per_prompt=1, generator=None, device="cpu", lat=None,
                 output_type=None, prompt_embeds=None, negative_prompt_embeds=None, pooled_prompt_embeds=None,
                 negative_pooled_prompt_embeds=None, use_graph=True, **kwargs):
        """base.py:828-850 for StableDiffusion3Pipeline (its default guidance 7.0; the reference
        passes 50 steps) -> the device flow-match loop and the VAE decode (see base generate)."""
        if self.pipeline is None:
            raise RuntimeError("The diffusion pipeline is not loaded. Please use `from_pretrained` or `from_quantized` first.")
        ctx, pooled = self._text_context(prompt, negative_prompt, prompt_embeds, negative_prompt_embeds,
                                         pooled_prompt_embeds, negative_pooled_prompt_embeds)
        if num_images_per_prompt > 1:
            b0 = ctx.shape[0] // 2
            r = num_images_per_prompt
            ctx = torch.cat([ctx[:b0].repeat_interleave(r, 0), ctx[b0:].repeat_interleave(r, 0)])
            pooled = torch.cat([pooled[:b0].repeat_interleave(r, 0), pooled[b0:].repeat_interleave(r, 0)])
        b = ctx.shape[0] // 2
        cin = self.pipeline.transformer.config.in_channels
        shape = (b, cin, height // 8, width // 8)
        if lat is None:
            lat = torch.randn(shape, generator=generator, dtype=torch.float32).to(torch.float16)
        loop = self.get_loop(b, height, width, num_inference_steps, guidance_scale, use_graph, ctx.shape[1])
        return self._decode(loop.run(lat.to(self.pipeline.device), ctx, pooled), output_type)

    @torch.no_grad()
    def run_sq_calibration(self, *a, **k):
        raise NotImplementedError("SmoothQuant calibration is UNet-only in the reference")


CLASS_MAP = {
    "StableDiffusionPipeline": StableDiffusion1_x,
    "StableDiffusionXLPipeline": StableDiffusionXL,
    "StableDiffusion3Pipeline": StableDiffusion3_5,
}


class AWQ:
    """Facade of the README (``AWQ.from_pretrained(model_id)``): dispatch on _class_name."""

    @staticmethod
    def from_pretrained(model_path, model_type=None, **kwargs):
        cls_name = load_config(model_path)["_class_name"]
        if cls_name not in CLASS_MAP:
            raise NotImplementedError(f"{cls_name} is not supported")
        return CLASS_MAP[cls_name].from_pretrained(model_path, model_type, **kwargs)

    @staticmethod
    def from_quantized(model_path, model_type=None, **kwargs):
        cls_name = load_config(model_path)["_class_name"]
        return CLASS_MAP[cls_name].from_quantized(model_path, model_type, **kwargs)
