"""Diffusion branches of AwqQuantizer (quantize/quantizer.py) and SqQuantizer
(quantize/quantizer_SQ.py): traverse the selected pipeline components, optionally fold
SmoothQuant scales into LayerNorm -> Linear groups, and swap every nn.Linear / nn.Conv2d for
WxAxLinear / WxAxConv2d.

Same constructor signature (positional order of quantizer.py:36-82), same traversal
(``MyTraversal``, quantizer.py:142-159), same per-layer decisions (quantizer.py:491-533):
  Linear -> WxAxLinear.from_float(weight_quant=weight_quant_type, act_quant='per_token',
            quantize_output=('k_proj'|'v_proj'|'q_proj' in child name), n_bits_W=w_bit,
            n_bits_A=a_bit, group_size_W=group_size)
  Conv2d -> WxAxConv2d.from_float(weight_quant=weight_quant_conv_type,
            act_quant=act_quant_conv_type, quantize_output=quantise_act,
            act_group_size=act_quant_conv_group_size, n_bits_W=w_bit, n_bits_A=a_bit)
Weight quantization runs on the GPU (libqdiff qd_weight_quant); the reference runs it on CPU
after moving the pipeline there (base.py:423) - the resulting fp16 buffers are bit-identical.

Intended-semantics fixes: the committed SQ source calls the
non-existent ``get_model_layers`` attribute (quantizer_SQ.py:1030) and the undefined name
``lin_and_conv_quantizelayers`` (:386); we implement what the committed .pyc does
(``get_model_layers_unet()`` and ``lin_and_conv_layers``).
"""
import torch
from torch import nn

from .calib import CalibrationSession
from .fake_quant import WxAxConv2d, WxAxLinear
from . import kernels as K


class MyTraversal:
    """quantizer.py:142-159: collect (parent, name, module) for every Linear / Conv2d."""

    def __init__(self):
        self.name = None
        self.parent = None
        self.lin_conv = []

    def traverse(self, name, module, parent):
        self.name = name
        self.parent = parent
        if isinstance(module, (nn.Linear, nn.Conv2d)):
            self.lin_conv.append((parent, name, module))
        for cname, child in module.named_children():
            if child is not None:
                self.traverse(cname, child, module)

    def get_lin_conv(self):
        return self.lin_conv


def _is_bmm_input(name):
    # quantizer.py:501 - substring test on the CHILD name only
    return "k_proj" in name or "v_proj" in name or "q_proj" in name


class AwqQuantizer:
    def __init__(self, awq_model, model, tokenizer, quantise_act, weight_quant_conv_type, weight_quant_type,
                 act_quant_conv_type, act_quant_conv_group_size, w_bit, wv_bit, a_bit, group_size, zero_point,
                 version, calib_data=None, split=None, text_column=None, duo_scaling=True,
                 modules_to_not_convert=None, export_compatible=False, quant_act=False, apply_clip=True,
                 applyScale=True, samples=512, processor=None, calib_data_type="", blocksize=512,
                 n_parallel_calib_samples=None, max_calib_samples=128, max_calib_seq_len=512,
                 max_chunk_memory=1024 * 1024 * 1024, LLM_ViT_serial=True, quantVision=False, quantText=True,
                 quantVisionProjection=False, quantTextProjection=False, quantUnet=True, quantTextEncoder=False,
                 quantVAE=False, quantTransformer=False, diffusion_model=False, codeBookQuantInd=False, **kwargs):
        self.awq_model = awq_model
        self.model = model
        self.tokenizer = tokenizer
        self.quantise_act = quantise_act
        self.weight_quant_conv_type = weight_quant_conv_type
        self.weight_quant_type = weight_quant_type
        self.act_quant_conv_type = act_quant_conv_type
        self.act_quant_conv_group_size = act_quant_conv_group_size
        self.w_bit = w_bit
        self.wv_bit = wv_bit
        self.a_bit = a_bit
        self.group_size = group_size
        self.zero_point = zero_point
        self.version = version
        self.modules_to_not_convert = modules_to_not_convert or []
        self.quantUnet = quantUnet
        self.quantTextEncoder = quantTextEncoder
        self.quantVAE = quantVAE
        self.quantTransformer = quantTransformer
        self.codeBookQuantInd = codeBookQuantInd
        self.diffusion_model = diffusion_model
        # this build's int8-MFMA W8A8 mode: per-output-channel int8 weights,
        # per-token (linear) / per-sample (conv) int8 activations on v_mfma_i32_16x16x64_i8
        self.int8_mfma = bool(kwargs.pop("int8_mfma", False))
        # this build's W4A8-fp8 mode for the SD3.5 transformer (per-token e4m3 activations)
        self.fp8_act = bool(kwargs.pop("fp8_act", False))
        # this build's AWQ scale + clip search for the UNet (awq_search.py; the reference keeps
        # it off for diffusion, quantizer.py:1050); apply_clip / duo_scaling as the reference's
        self.awq_search = bool(kwargs.pop("awq_search", False))
        self.apply_clip = apply_clip
        self.duo_scaling = duo_scaling
        self.search_report = None
        self.calib_kwargs = kwargs
        if not diffusion_model:
            raise NotImplementedError("the LLM/VLM AWQ path is out of scope (SURVEY.md §2); diffusion_model=True only")
        self.modules, self.module_kwargs, self.inps = self.init_quant()

    MyTraversal = MyTraversal

    def init_quant(self, *a, **k):
        """Diffusion branch of init_quant (quantizer.py:1049-1091); calibration is off (:1050)."""
        modules = {"unet": [], "text_encoder": [], "vae": [], "transformer": []}
        if self.quantUnet:
            modules["unet"] = self.awq_model.get_model_layers_unet()
        if self.quantTextEncoder:
            modules["text_encoder"] = self.awq_model.get_model_layers_te()
        if self.quantVAE:
            modules["vae"] = self.awq_model.get_model_layers_vae()
        if self.quantTransformer:
            modules["transformer"] = self.awq_model.get_model_layers_transformers()
        return modules, [], []

    def _swap_components(self):
        """quantizer.py:386-425: per component, per top-level child with parameters, swap."""
        for key, comps in self.modules.items():
            if not comps:
                continue
            for k, module_list in enumerate(comps):
                root = self.awq_model.get_root(key, k)
                self.awq_model.set_quantized_components(f"{key}_{k + 1}" if len(comps) > 1 and k > 0 else key)
                for name, mod in module_list:
                    try:
                        next(mod.parameters())
                    except StopIteration:
                        continue  # parameterless child (quantizer.py:407-410)
                    trav = self.MyTraversal()
                    trav.traverse(name, mod, root)
                    self._apply_quant_fake_act(mod, trav.get_lin_conv(), self.w_bit)

    def quantize(self, debugSavePath="", debugPlot=False):
        if self.awq_search:
            if not self.quantUnet or not self.duo_scaling:
                raise NotImplementedError("awq_search: UNet transformer blocks with duo_scaling only")
            from .awq_search import run_awq_search
            self.search_report = run_awq_search(self.awq_model, self.w_bit, self.group_size,
                                                calibration=self.calib_kwargs.get("calibration"),
                                                clip=self.apply_clip)
        self._swap_components()

    @torch.no_grad()
    def _apply_quant_fake_act(self, module, named_linears, bitWidth, debugStruct=None, debug=False):
        """Diffusion branch of quantizer.py:491-533."""
        for parent, name, layer in named_linears:
            i8 = getattr(self, "int8_mfma", False) and bitWidth == 8
            if isinstance(layer, nn.Linear):
                fake = WxAxLinear.from_float(layer, weight_quant=self.weight_quant_type, act_quant="per_token",
                                             quantize_output=_is_bmm_input(name), n_bits_W=bitWidth,
                                             n_bits_A=self.a_bit, group_size_W=self.group_size,
                                             codeBookQuantInd=self.codeBookQuantInd,
                                             int8_mfma=i8 and layer.in_features % 64 == 0,
                                             fp8_act=getattr(self, "fp8_act", False))
                setattr(parent, name, fake)
            elif isinstance(layer, nn.Conv2d):
                fake = WxAxConv2d.from_float(layer, weight_quant=self.weight_quant_conv_type,
                                             act_quant=self.act_quant_conv_type, quantize_output=self.quantise_act,
                                             act_group_size=self.act_quant_conv_group_size, n_bits_W=bitWidth,
                                             n_bits_A=self.a_bit, codeBookQuantInd=self.codeBookQuantInd,
                                             int8_mfma=i8)
                setattr(parent, name, fake)


class SqQuantizer(AwqQuantizer):
    """SmoothQuant diffusion branch (quantizer_SQ.py:323-391, 395-431, 1025-1070)."""

    alpha = 0.80  # quantizer_SQ.py:349

    def quantize(self, debugSavePath="", debugPlot=False):
        blocks = self.awq_model.get_smoothing_blocks()
        calib = self.calib_kwargs.get("calibration", None)
        session = CalibrationSession(blocks)
        session.attach()
        try:
            self.awq_model.run_sq_calibration(**(calib or {}))
        finally:
            session.detach()
        for block_name, block in blocks.items():
            for group in self.awq_model.get_layers_for_scaling_unet(block, session.hooks[block_name]):
                self.smooth_ln_fcs(group["prev_op"], group["layers"], group["activations_max"][0], alpha=self.alpha)
        session.clear()
        self._swap_components()

    @torch.no_grad()
    def smooth_ln_fcs(self, ln, fcs, act_scales, model_type="transformers", alpha=0.5):
        """quantizer_SQ.py:395-431 on device: s = clamp(a^alpha / max_fc|W|^(1-alpha), 1e-5);
        ln.w /= s; ln.b /= s; fc.W *= s."""
        if not isinstance(fcs, list):
            fcs = [fcs]
        for fc in fcs:
            assert ln.weight.numel() == fc.in_features == act_scales.numel()
        lb = ln.bias if getattr(ln, "bias", None) is not None else None
        return K.smooth_fold(ln.weight.data, lb.data if lb is not None else None, [fc.weight.data for fc in fcs],
                             act_scales, alpha=alpha)
