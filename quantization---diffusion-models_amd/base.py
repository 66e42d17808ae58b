"""BaseAWQForDiffusion: the public from_pretrained() / quantize() / generate() /
save_quantized() / from_quantized() surface of models/base.py:120-850, on MI355X.

Divergences from the reference, all deliberate and documented in DESIGN.md:
* the pipeline lives on the GPU; quantize() quantizes weights there (the reference moves the
  pipeline to CPU first, base.py:423) - the fp16 buffers are bit-identical;
* generate() honours height / width / num_inference_steps / guidance_scale (the reference
  passes only prompt, 50 steps, generator, latents, output_type: base.py:848).  The defaults
  equal the reference's effective values, so default calls match;
* prompts are encoded by the pipeline's CLIP text encoder(s) and latents decoded by its VAE on
  device (clip.py, vae.py); pipelines without them map prompts to synthetic embeddings and
  return latents only; SD3 runs without T5 (zero T5 features, as diffusers does without
  text_encoder_3);
* from_pretrained() never contacts the hub; the hard-coded access token default of
  base.py:188 is not reproduced.
"""
import json
import os
from typing import List, Optional, Union

import torch
from torch import nn

from .config import AwqConfig
from .fake_quant import WxAxConv2d, WxAxLinear
from .pipeline import make_loop, synthetic_text_embeddings
from .pipeline_io import QDiffPipeline, load_config, load_pipeline
from .quantizer import AwqQuantizer, MyTraversal, SqQuantizer

QUANTISABLE_COMPONENTS = ["unet", "text_encoder", "vae", "transformer"]


class _HybridMethod:
    """Callable on the class (constructs) or on an instance (reloads in place), because the
    reference defines from_quantized as an instance method (base.py:736)."""

    def __init__(self, f):
        self.f = f

    def __get__(self, obj, cls):
        def bound(*a, **k):
            return self.f(obj if obj is not None else cls, *a, **k)
        return bound


class BaseAWQForDiffusion(nn.Module):
    def __init__(self, pipeline, model_type, is_quantized, config, quant_config):
        super().__init__()
        self.model_type = model_type
        self.is_quantized = is_quantized
        self.config = config
        self.pipeline = pipeline
        self.search_result = None
        self.quant_config = quant_config
        self._loops = {}

    def to(self, device):
        if self.pipeline is None:
            raise RuntimeError("The diffusion pipeline is not loaded. Please use `from_pretrained` or `from_quantized` first.")
        self.pipeline.to(device)
        self._loops = {}
        return self

    # ---------------------------------------------------------------- loading
    @classmethod
    def from_pretrained(cls, model_path, model_type=None, torch_dtype=torch.float16, trust_remote_code=True,
                        safetensors=True, device_map="auto", download_kwargs=None, low_cpu_mem_usage=True,
                        use_cache=False, refiner_path=None, token=None, device="cuda", seed=0, scheduler=None,
                        **model_init_kwargs):
        """base.py:143-212 (local directories / synthetic names only; fp16 always, as base.py:199).
        The scheduler is the checkpoint's own (scheduler/scheduler_config.json: PNDM for SD1.5, as
        DiffusionPipeline.from_pretrained builds it); scheduler="ddim" / "pndm" overrides it."""
        pipe = load_pipeline(model_path, device=device, seed=seed, scheduler=scheduler)
        quant_config = AwqConfig.from_pretrained(model_path, is_diffusion_model=True)
        config = load_config(model_path)
        model_type = config["_class_name"]
        return cls(pipe, model_type, is_quantized=False, config=config, quant_config=quant_config,
                   refiner_path=refiner_path, access_token=token)

    # ---------------------------------------------------------------- quantize
    @torch.no_grad()
    def quantize(self, tokenizer=None, quant_config={}, calib_data="pileval", split="train", text_column="text",
                 duo_scaling=True, export_compatible=False, quant_act=False, apply_clip=True, applyScale=True,
                 samples=512, calib_data_type="", blocksize=512, n_parallel_calib_samples=None,
                 max_calib_samples=128, max_calib_seq_len=512, max_chunk_memory=1024 * 1024 * 1024,
                 quantizer_cls=AwqQuantizer, quantType="awq", LLM_ViT_serial=False, quantVision=False,
                 quantText=True, quantVisionProjection=False, quantTextProjection=False, quantUnet=False,
                 quantTextEncoder=False, quantVAE=False, quantTransformer=False, diffusion_model=True,
                 codeBookQuantInd=False, debugPlot=False, debugAttentionMap=False, debugSavePath="",
                 calibration=None, int8_mfma=False, awq_search=False, fp8_act=False, **kwargs):
        """base.py:215-528.  quantType 'awq' = RTN swap; 'sq' = SmoothQuant fold + swap.
        int8_mfma=True (this build, w_bit 8): the int8-MFMA W8A8 mode instead of the reference's
        fake-quant arithmetic (re-granularized, tolerance-based parity).
        fp8_act=True (w_bit 4, group 128; the SD3.5 transformer): per-token e4m3 activations on
        the fp8 MFMA, BASELINE config C5's "fp8 activations on CDNA4".
        awq_search=True (quantType 'awq'): the AWQ activation-aware scale search and weight-clip
        search on the UNet's transformer blocks before the RTN swap (awq_search.py; calibration=
        as run_sq_calibration's keywords)."""
        if quant_act and quant_config.get("version", "fake_act").lower() != "fake_act":
            print("With activation quantization set to True, you can only use the fake quant kernel fake_act! "
                  "Changing to that....")
            quant_config["version"] = "fake_act"
        self.quant_config = AwqConfig.from_dict(quant_config)
        if hasattr(self, "modules_to_not_convert"):
            self.quant_config.modules_to_not_convert = self.modules_to_not_convert
        qc = self.quant_config
        common = dict(modules_to_not_convert=qc.modules_to_not_convert, export_compatible=export_compatible,
                      quant_act=quant_act, apply_clip=apply_clip, applyScale=applyScale, samples=samples,
                      calib_data_type=calib_data_type, blocksize=blocksize, quantUnet=quantUnet,
                      quantTextEncoder=quantTextEncoder, quantVAE=quantVAE, quantTransformer=quantTransformer,
                      diffusion_model=True, codeBookQuantInd=codeBookQuantInd, int8_mfma=int8_mfma,
                      fp8_act=fp8_act)
        args = (self, None, None, qc.quantize_act, qc.weight_quant_conv_type, qc.weight_quant_type,
                qc.act_quant_conv_type, qc.act_quant_conv_group_size, qc.w_bit, qc.wv_bit, qc.a_bit,
                qc.q_group_size, qc.zero_point, qc.version, calib_data, split, text_column, duo_scaling)
        if quantType.lower() == "awq":
            self.quantizer = quantizer_cls(*args, **common, awq_search=awq_search, calibration=calibration, **kwargs)
        elif quantType.lower() == "sq":
            self.quantizer = SqQuantizer(*args, **common, calibration=calibration)
        else:
            raise NotImplementedError("Only awq and sq are supported for now.")
        self.quantizer.quantize(debugSavePath, debugPlot)
        self.is_quantized = True
        self.int8_mfma = bool(int8_mfma)
        self.fp8_act = bool(fp8_act)
        self._loops = {}

    # ---------------------------------------------------------------- generate
    def _has_text_encoder(self):
        return "text_encoder" in self.pipeline.component_names()

    def _text_context(self, prompt, negative_prompt, prompt_embeds, negative_prompt_embeds):
        """StableDiffusionPipeline.encode_prompt: [negative; positive] CLIP last hidden states
        (the negative prompt defaults to ""); pipelines without a text encoder map prompt strings
        to deterministic synthetic embeddings."""
        dim = self.pipeline.unet.config.cross_attention_dim
        dev = self.pipeline.device
        pipe = self.pipeline
        te = self._has_text_encoder()
        if prompt_embeds is None:
            prompts = [prompt] if isinstance(prompt, str) else list(prompt)
            prompt_embeds = (pipe.text_encoder.encode(pipe.tokenizer(prompts))[0] if te else
                             synthetic_text_embeddings(prompts, dim=dim, device=dev))
        if negative_prompt_embeds is None:
            b = prompt_embeds.shape[0]
            neg = negative_prompt if negative_prompt is not None else ""
            negs = [neg] * b if isinstance(neg, str) else list(neg)
            negative_prompt_embeds = (pipe.text_encoder.encode(pipe.tokenizer(negs, max_length=prompt_embeds.shape[1]))[0]
                                      if te else synthetic_text_embeddings(negs, seq_len=prompt_embeds.shape[1], dim=dim,
                                                                           device=dev))
        return torch.cat([negative_prompt_embeds.to(dev), prompt_embeds.to(dev)]).to(torch.float16).contiguous()

    def _decode(self, latents, output_type):
        """output_type "latent": the latents; otherwise VAE decode + VaeImageProcessor.postprocess
        (None -> "np", as diffusers treats it; "pt" / "pil" as diffusers)."""
        if output_type == "latent":
            return latents
        if output_type not in (None, "np", "pt", "pil"):
            raise ValueError(f"output_type {output_type!r}: one of 'latent', 'np', 'pt', 'pil' (None = 'np')")
        if "vae" not in self.pipeline.component_names():
            raise RuntimeError("this pipeline has no VAE (vae/ directory): use output_type='latent'")
        from . import kernels as K
        c = latents.shape[1]
        return self.pipeline.vae.decode_images(K.nchw_to_nhwc(latents.contiguous(), (c + 7) // 8 * 8),
                                               output_type or "np")

    def get_loop(self, batch, height, width, steps, guidance, use_graph=True):
        key = (batch, height, width, steps, float(guidance), use_graph)
        if key not in self._loops:
            self._loops[key] = make_loop(self.pipeline.unet, batch, height, width, steps, guidance,
                                         self.pipeline.device, use_graph, self.pipeline.scheduler_config)
        return self._loops[key]

    @torch.no_grad()
    def generate(self, prompt=None, height=512, width=512, num_inference_steps=50, guidance_scale=7.5,
                 negative_prompt=None, num_images_per_prompt=1, generator=None, device="cpu", lat=None,
                 output_type=None, prompt_embeds=None, negative_prompt_embeds=None, use_graph=True, **kwargs):
        """base.py:828-850 -> the device denoising loop, then the VAE decode (output_type None:
        float32 numpy images [B, H, W, 3] as the reference's pipeline call returns; "latent":
        the latents [B, 4, h, w] fp16)."""
        if self.pipeline is None:
            raise RuntimeError("The diffusion pipeline is not loaded. Please use `from_pretrained` or `from_quantized` first.")
        ctx = self._text_context(prompt, negative_prompt, prompt_embeds, negative_prompt_embeds)
        if num_images_per_prompt > 1:
            b0 = ctx.shape[0] // 2
            ctx = torch.cat([ctx[:b0].repeat_interleave(num_images_per_prompt, 0),
                             ctx[b0:].repeat_interleave(num_images_per_prompt, 0)])
        b = ctx.shape[0] // 2
        cin = self.pipeline.unet.config.in_channels
        shape = (b, cin, height // 8, width // 8)
        if lat is None:
            lat = torch.randn(shape, generator=generator, dtype=torch.float32).to(torch.float16)
        loop = self.get_loop(b, height, width, num_inference_steps, guidance_scale, use_graph)
        return self._decode(loop.run(lat.to(self.pipeline.device), ctx), output_type)

    # ---------------------------------------------------------------- save / load
    def save_quantized(self, save_dir, safetensors=True, shard_size="5GB", export_compatible=False, quant_act=False,
                       awq_export=True):
        """base.py:530-582: pipeline files + quantization_config in each quantized component's
        config.json + quant_components.json (reference-compatible fp16 dequantized buffers), plus
        this build's integer formats (export.py): every linear's codes / scales and every conv's
        codes (the reference's per-(Co, Ci, kh) granularity, and the int8-MFMA mode's
        per-output-channel codes) in <denoiser>/qdiff_codes.safetensors, the 4-bit linears also in
        the AWQ GEMM layout (<denoiser>/awq_gemm.safetensors: qweight / qzeros / scales, the
        reference's utils/quant_utils.py / packing_utils.py order), and the full quant config
        (qdiff_quant.json)."""
        from safetensors.torch import save_file
        save_dir = save_dir[:-1] if save_dir.endswith("/") else save_dir
        os.makedirs(save_dir, exist_ok=True)
        self.pipeline.save_pretrained(save_dir, safe_serialization=safetensors)
        for comp in self.quantized_components:
            cpath = os.path.join(save_dir, comp, "config.json")
            if not os.path.exists(cpath):
                continue
            with open(cpath) as f:
                cfg = json.load(f)
            cfg["quantization_config"] = self.quant_config.to_transformers_dict()
            with open(cpath, "w") as f:
                json.dump(cfg, f, indent=2)
        with open(os.path.join(save_dir, "quant_components.json"), "w") as f:
            json.dump(self.quantized_components, f, indent=2)
        with open(os.path.join(save_dir, "qdiff_quant.json"), "w") as f:
            json.dump(dict(self.quant_config.full_dict(), int8_mfma=bool(getattr(self, "int8_mfma", False)),
                           fp8_act=bool(getattr(self, "fp8_act", False))), f, indent=2)
        from .export import awq_pack_linear, conv_codes, packed_nibbles_to_codes
        codes, awq = {}, {}
        for name, m in self.pipeline.denoiser.named_modules():
            if isinstance(m, WxAxLinear) and m.gemm_weight()[1] != "f16":
                codes[f"{name}.qcodes"] = m.qcodes.detach().cpu().contiguous()
                codes[f"{name}.qscales"] = m.qscales.detach().cpu().contiguous()
                codes[f"{name}.qmeta"] = torch.tensor([m.qgroup, m.n_bits_W, int(m.int8_mfma)], dtype=torch.int32)
                if awq_export and m.qfmt == "i4":
                    c = packed_nibbles_to_codes(m.qcodes, m.in_features)
                    for k, v in awq_pack_linear(c, m.qscales, m.qgroup).items():
                        awq[f"{name}.{k}"] = v.detach().cpu().contiguous()
            elif isinstance(m, WxAxConv2d):
                i8 = m.i8_operand()
                if i8 is not None:
                    codes[f"{name}.i8_w"] = i8[0].detach().cpu().contiguous()
                    codes[f"{name}.i8_sw"] = i8[1].detach().cpu().contiguous()
                elif m.weight_quant_name == "per_channel" and getattr(m, "n_bits_W", 16) <= 8:
                    cc, cs = conv_codes(m.weight.detach(), m.n_bits_W)
                    codes[f"{name}.conv_qcodes"] = cc.cpu().contiguous()
                    codes[f"{name}.conv_qscales"] = cs.cpu().contiguous()
        sub = os.path.join(save_dir, self.pipeline.denoiser_name)
        if codes:
            save_file(codes, os.path.join(sub, "qdiff_codes.safetensors"))
        if awq:
            save_file(awq, os.path.join(sub, "awq_gemm.safetensors"))

    def _load_quantized_modules(self, module, bitWidth=4, group_size=128, act_bits=16, full_config=None):
        return load_quantized_modules(module, bitWidth, group_size, act_bits, full_config)


    @_HybridMethod
    def from_quantized(self_or_cls, model_path, model_type=None, model_filename="", torch_dtype=torch.float16,
                       safetensors=True, fuse_layers=True, use_ipex=False, device_map="balanced", max_memory=None,
                       offload_folder=None, download_kwargs=None, device="cuda"):
        """base.py:736-826 (usable on an instance, as in the reference, or on the class)."""
        from safetensors.torch import load_file
        from .mmdit import MMDiTConfig, SD3Transformer2DModel
        from .unet import UNet2DConditionModel, UNetConfig
        with open(os.path.join(model_path, "quant_components.json")) as f:
            comps = json.load(f)
        with open(os.path.join(model_path, "model_index.json")) as f:
            cls_name = json.load(f)["_class_name"]
        sub = "transformer" if "transformer" in comps else "unet"
        with open(os.path.join(model_path, sub, "config.json")) as f:
            ucfg_d = json.load(f)
        if sub == "transformer":
            net = SD3Transformer2DModel(MMDiTConfig.from_diffusers(ucfg_d)).half().to(device)
        else:
            net = UNet2DConditionModel(UNetConfig.from_diffusers(ucfg_d)).half().to(device)
        qc = ucfg_d["quantization_config"]
        full = None
        fpath = os.path.join(model_path, "qdiff_quant.json")
        if os.path.exists(fpath):
            with open(fpath) as f:
                full = json.load(f)
        if full:
            from dataclasses import fields as _fields
            qcfg = AwqConfig(**{f.name: full[f.name] for f in _fields(AwqConfig) if f.name in full})
        else:
            qcfg = AwqConfig(**AwqConfig.from_transformers_dict(AwqConfig, qc))
        load_quantized_modules(net, bitWidth=qc["bits"], group_size=qc["group_size"], act_bits=qc["act_bits"],
                               full_config=full)
        sd = load_file(os.path.join(model_path, sub, "diffusion_pytorch_model.safetensors"))
        net.load_state_dict({k: v.to(device) for k, v in sd.items()}, strict=True)
        cpath = os.path.join(model_path, sub, "qdiff_codes.safetensors")
        codes = load_file(cpath) if os.path.exists(cpath) else {}
        apath = os.path.join(model_path, sub, "awq_gemm.safetensors")
        awq = load_file(apath) if os.path.exists(apath) and not codes else {}
        int8 = bool((full or {}).get("int8_mfma", False))
        fp8 = bool((full or {}).get("fp8_act", False))
        for name, m in net.named_modules():
            if isinstance(m, WxAxConv2d):
                if f"{name}.i8_w" in codes:
                    _attach_conv_i8(m, codes[f"{name}.i8_w"].to(device), codes[f"{name}.i8_sw"].to(device))
                continue
            if not isinstance(m, WxAxLinear):
                continue
            if f"{name}.qcodes" in codes:
                meta = codes[f"{name}.qmeta"].tolist()
                g, nb = meta[0], meta[1]
                m.qcodes = codes[f"{name}.qcodes"].to(device)
                m.qscales = codes[f"{name}.qscales"].to(device)
                m.qgroup, m.n_bits_W = g, nb
                m.qfmt = "i4" if nb <= 4 else "i8"
                m._codes_ver = (m.weight.data_ptr(), m.weight._version)
                m.int8_mfma = bool(meta[2]) if len(meta) > 2 else False
            elif f"{name}.qweight" in awq:
                from .export import awq_unpack_linear
                from .kernels import pack_int4
                c, sc = awq_unpack_linear(awq[f"{name}.qweight"], awq[f"{name}.qzeros"], awq[f"{name}.scales"],
                                          qc["group_size"] if m.in_features % qc["group_size"] == 0 else
                                          m.in_features // awq[f"{name}.scales"].shape[0])
                # kept only if the codes dequantize to the stored fp16 buffer bit for bit (a foreign
                # or mismatched AWQ file would otherwise make the GEMM operand differ from `weight`)
                g = m.in_features // sc.shape[1]
                c, sc = c.to(device), sc.to(device)
                deq = (c.float() * sc.float().repeat_interleave(g, dim=1)).to(torch.float16)
                if not (torch.equal(deq.float(), m.weight.float()) and m.set_codes(c, sc, g, 4)):
                    m.drop_codes()  # the fp16 buffer (the reference's own operand)
            else:
                # a reference-written checkpoint holds only the dequantized fp16 buffers: re-derive
                # the integer codes and keep them only if they reproduce the buffer bit for bit
                rederive_codes(m, qc["bits"], qc["group_size"])
                m.int8_mfma = int8 and m.qfmt == "i8" and m.qgroup == m.in_features
            if fp8 and m.qfmt == "i4" and m.gemm_weight()[1] == "i4":
                from .export import packed_nibbles_to_codes
                m.set_fp8(packed_nibbles_to_codes(m.qcodes, m.in_features), m.qscales, m.qgroup, m.n_bits_W)
        from .pipeline_io import _local_aux, load_scheduler_config
        aux = dict(lazy=_local_aux(model_path), scheduler_config=load_scheduler_config(model_path))
        if sub == "transformer":
            pipe = QDiffPipeline(transformer=net, class_name=cls_name, config={"_class_name": cls_name}, **aux)
        else:
            pipe = QDiffPipeline(net, cls_name, config={"_class_name": cls_name}, **aux)
        if isinstance(self_or_cls, type):
            obj = self_or_cls(pipe, cls_name, is_quantized=True, config={"_class_name": cls_name}, quant_config=qcfg)
        else:
            obj = self_or_cls
            obj.pipeline = pipe
            obj.is_quantized = True
            obj.quant_config = qcfg
            obj._loops = {}
        obj.quantized_components = comps
        obj.int8_mfma = bool((full or {}).get("int8_mfma", False))
        obj.fp8_act = fp8
        return obj


@torch.no_grad()
def _attach_conv_i8(m, codes, sw):
    """int8-MFMA conv codes from a checkpoint; kept only if they dequantize to the stored buffer."""
    co, ci, kh, kw = m.weight.shape
    deq = (codes.float() * sw[:, None, None, None]).to(torch.float16)[..., :ci].permute(0, 3, 1, 2)
    if not torch.equal(deq.float(), m.weight.float()):  # value-equal (-0.0 of the fp16 buffer)
        return False
    m.i8_w, m.i8_sw = codes.contiguous(), sw.contiguous()
    m._i8_ver = (m.weight.data_ptr(), m.weight._version)
    m._fq_saved = (m.quantise_act, m.output_quant_name, m.output_quant)
    m.quantise_act = False
    m.output_quant_name = "None"
    m.output_quant = lambda x: x
    return True


@torch.no_grad()
def rederive_codes(m, n_bits, group_size):
    """Integer codes of a loaded WxAxLinear whose checkpoint stored only ``weight`` (the
    reference's format, base.py:530-582): RTN of the dequantized buffer with the same bits and
    group (shrink rule included).  Attached only when dequantizing them gives back exactly the
    stored buffer, so the GEMM operand is unchanged; otherwise the fp16 buffer stays the operand."""
    from .fake_quant import quantize_weight_absmax_codes, shrink_group
    if n_bits > 8 or m.in_features % 64 != 0:
        return False
    try:
        g = shrink_group(m.in_features, group_size) if group_size > 0 else m.in_features
    except ZeroDivisionError:
        return False
    codes, scales, wdq, g = quantize_weight_absmax_codes(m.weight, n_bits, g)
    if not torch.equal(wdq.view(torch.int16), m.weight.view(torch.int16)):
        return False
    return m.set_codes(codes, scales, g, n_bits)


def load_quantized_modules(module, bitWidth=4, group_size=128, act_bits=16, full_config=None):
    """base.py:658-692: init_only WxAx modules in place of every Linear / Conv2d.  Without our
    qdiff_quant.json (a reference checkpoint) conv layers get quantize_output=True and
    per_channel act quant, exactly as base.py:680-690 forces."""
    for name, child in module.named_children():
        trav = MyTraversal()
        trav.traverse(name, child, module)
        for parent, lname, layer in trav.get_lin_conv():
            qbmm = "k_proj" in lname or "v_proj" in lname or "q_proj" in lname
            if isinstance(layer, nn.Linear):
                fake = WxAxLinear.from_float(layer, init_only=True, weight_quant="group", act_quant="per_token",
                                             quantize_output=qbmm, n_bits_W=bitWidth, n_bits_A=act_bits,
                                             group_size_W=group_size)
            else:
                if full_config is not None:
                    fake = WxAxConv2d.from_float(layer, init_only=True,
                                                 weight_quant=full_config["weight_quant_conv_type"],
                                                 act_quant=full_config["act_quant_conv_type"],
                                                 act_group_size=full_config["act_quant_conv_group_size"],
                                                 quantize_output=full_config["quantize_act"],
                                                 n_bits_W=bitWidth, n_bits_A=act_bits)
                else:
                    fake = WxAxConv2d.from_float(layer, init_only=True, weight_quant="per_channel",
                                                 act_quant="per_channel", n_bits_W=bitWidth, n_bits_A=act_bits,
                                                 quantize_output=True)
            setattr(parent, lname, fake)
