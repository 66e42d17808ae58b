"""Fake-quant operators and the WxAxLinear / WxAxConv2d drop-in modules, on MI355X.

Mirrors /root/reference/quantize/fake_quant.py: same function and class names, the same
``from_float`` keyword surface, the same ``weight`` / ``bias`` fp16 buffers (so ``state_dict``
keys equal nn.Linear / nn.Conv2d keys and hold the dequantized values bit-for-bit), the same
``ValueError`` on an unknown granularity and the same group-size shrink rule.  Every
computation runs in libqdiff HIP kernels; CPU tensors are rejected (there is no CPU path in
the product - the CPU restatement lives in ``oracle/`` and is test infrastructure).

Beyond the reference, a quantized Linear also keeps its integer codes (int8, or int4 packed
two per byte) and fp16 group scales as non-persistent buffers; the forward GEMM dequantizes
them while staging the weight tile into LDS (``qd_linear_fwd`` with QD_WFMT_I8/I4), which
yields exactly the stored fp16 weight values (half(q * s)).
"""
from functools import partial

import torch
from torch import nn

from . import kernels as K


def _need_gpu(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the MI355X fake-quant path needs a HIP tensor (got {t.device}); "
                           "there is no CPU fallback in the product path")


def shrink_group(k, group_size, step=32):
    """``while K % g: g -= 32`` (fake_quant.py:33-37); g reaching 0 raises like the reference."""
    g = group_size
    while k % g != 0:
        g -= step
        if g == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
    return g


def per_group_size(h, w, group_size):
    """``while H % g or W % g: g -= 2`` (fake_quant.py:138-139)."""
    g = group_size
    while h % g != 0 or w % g != 0:
        g -= 2
        if g == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
    return g


# ------------------------------------------------------------------ weight quantizers
@torch.no_grad()
def quantize_weight_absmax_codes(w, n_bits=8, group_size=0):
    """Codes / scales / dequantized weight of quantize_weight_absmax (fake_quant.py:21-84).
    Returns (codes int8 [N, K], scales fp16 [N, K/g], w_dq fp16 [N, K], g)."""
    _need_gpu(w, "quantize_weight_absmax")
    shape = w.shape
    if group_size > 0:
        g = shrink_group(shape[-1], group_size)
    else:
        g = shape[-1]
    w2 = w.detach().to(torch.float16).contiguous().reshape(-1, shape[-1])
    if w2.dim() != 2 or (group_size <= 0 and w.dim() != 2):
        raise AssertionError("w.dim() == 2")  # fake_quant.py:41
    codes, scales, wdq = K.weight_quant(w2, g, n_bits)
    if codes is not None:  # None above 8 bits: dequantized weight only
        codes = codes.reshape(shape)
    return codes, scales.reshape(*shape[:-1], shape[-1] // g), wdq.reshape(shape), g


@torch.no_grad()
def quantize_weight_absmax(w, n_bits=8, group_size=0, codeBookQuantInd=False, debugPath=[], debug=False):
    """fake_quant.py:21-84.  The codebook branch (codeBookQuantInd=True) is out of scope."""
    if codeBookQuantInd:
        raise NotImplementedError("codebook weight quantization (genCodeBook.py) is out of scope")
    if group_size <= 0 and w.dim() != 2:
        raise AssertionError("w.dim() == 2")
    _, _, wdq, _ = quantize_weight_absmax_codes(w, n_bits, group_size)
    return wdq


@torch.no_grad()
def quantize_weight_per_channel_absmax(w, n_bits=8):
    """fake_quant.py:86-93: scale per row of the LAST dim (conv: per (Co, Ci, kh))."""
    _need_gpu(w, "quantize_weight_per_channel_absmax")
    shape = w.shape
    w2 = w.detach().to(torch.float16).contiguous().reshape(-1, shape[-1])
    _, _, wdq = K.weight_quant(w2, shape[-1], n_bits, want_codes=False, want_scales=False)
    return wdq.reshape(shape).to(w.dtype)


@torch.no_grad()
def quantize_weight_per_tensor_absmax(w, n_bits=8):
    """fake_quant.py:96-105."""
    _need_gpu(w, "quantize_weight_per_tensor_absmax")
    w2 = w.detach().to(torch.float16).contiguous().reshape(1, -1)
    _, _, wdq = K.weight_quant(w2, w2.shape[1], n_bits, want_codes=False, want_scales=False)
    return wdq.reshape(w.shape).to(w.dtype)


# ------------------------------------------------------------------ activation quantizers
@torch.no_grad()
def quantize_activation_per_token_absmax(t, n_bits=8):
    """fake_quant.py:108-118."""
    _need_gpu(t, "quantize_activation_per_token_absmax")
    return K.act_fakequant(t.contiguous().to(torch.float16), "per_token", n_bits).to(t.dtype)


@torch.no_grad()
def quantize_activation_per_channel_absmax(t, n_bits=8):
    """fake_quant.py:123-131 (NCHW, scale per (n, c) over H, W)."""
    _need_gpu(t, "quantize_activation_per_channel_absmax")
    return K.act_fakequant(t.contiguous().to(torch.float16), "per_channel", n_bits, layout=K.NCHW).to(t.dtype)


@torch.no_grad()
def quantize_activation_per_channel_group_absmax(t, group_size=128, n_bits=8):
    """fake_quant.py:133-153 (g x g spatial patches; g shrinks by 2 until it divides H and W)."""
    _need_gpu(t, "quantize_activation_per_channel_group_absmax")
    g = per_group_size(t.shape[2], t.shape[3], group_size)
    return K.act_fakequant(t.contiguous().to(torch.float16), "per_group", n_bits, layout=K.NCHW, group=g)


@torch.no_grad()
def quantize_activation_per_tensor_absmax(t, n_bits=8):
    """fake_quant.py:157-167."""
    _need_gpu(t, "quantize_activation_per_tensor_absmax")
    return K.act_fakequant(t.contiguous().to(torch.float16), "per_tensor", n_bits).to(t.dtype)


def _act_quant_fn(name, n_bits, group=1):
    if name == "per_token":
        return partial(quantize_activation_per_token_absmax, n_bits=n_bits)
    if name == "per_tensor":
        return partial(quantize_activation_per_tensor_absmax, n_bits=n_bits)
    if name == "per_channel":
        return partial(quantize_activation_per_channel_absmax, n_bits=n_bits)
    if name == "per_group":
        return partial(quantize_activation_per_channel_group_absmax, n_bits=n_bits, group_size=group)
    raise ValueError(f"Invalid act_quant: {name}")


def _identity(x):
    return x


# ------------------------------------------------------------------ modules
class WxAxLinear(nn.Module):
    """Drop-in for nn.Linear with fake-quantized weight (fake_quant.py:170-261).

    Buffers ``weight`` (fp16 dequantized, [out, in]) and ``bias`` as in the reference.
    Non-persistent ``qcodes`` / ``qscales`` hold the integer form used by the fused GEMM.
    """

    def __init__(self, in_features, out_features, bias=True, weight_quant="per_channel",
                 act_quant="per_token", quantize_output=False, n_bits_A=16, q_act=False):
        super().__init__()
        self.quantize_act = q_act
        self.in_features = in_features
        self.out_features = out_features
        self.n_bits_A = n_bits_A
        self.register_buffer("weight", torch.zeros(out_features, in_features, dtype=torch.float16))
        if bias:
            self.register_buffer("bias", torch.zeros(out_features, dtype=torch.float16))
        else:
            self.register_buffer("bias", None)
        self.register_buffer("qcodes", None, persistent=False)
        self.register_buffer("qscales", None, persistent=False)
        self.qfmt = "f16"
        self.qgroup = 0
        self.n_bits_W = 16
        self.int8_mfma = False  # int8-MFMA W8A8 mode (per-row int8 codes x per-token int8 activations)
        self.fp8_act = False    # W4A8-fp8 mode (W4 group-128 codes as e4m3 x per-token e4m3 activations)
        self.weight_quant_name = weight_quant
        if act_quant == "per_token":
            self.act_quant_name = "per_token"
        elif act_quant == "per_tensor":
            self.act_quant_name = "per_tensor"
        else:
            raise ValueError(f"Invalid act_quant: {act_quant}")  # fake_quant.py:197-198
        self.act_quant = _act_quant_fn(self.act_quant_name, n_bits_A)
        if quantize_output:
            self.output_quant_name = self.act_quant_name
            self.output_quant = self.act_quant
        else:
            self.output_quant_name = "None"
            self.output_quant = _identity

    def _apply(self, fn, *args, **kwargs):
        """Module.to / .cuda / .half: codes that describe ``weight`` before the move still describe
        it after (same values, new storage), so they are re-stamped instead of being dropped as
        stale (which would silently leave the int8-MFMA / fp8 mode); the fp8 operand, held outside
        the buffer set, follows the weight's device."""
        codes_fresh = self.qcodes is not None and \
            getattr(self, "_codes_ver", None) == (self.weight.data_ptr(), self.weight._version)
        f8 = getattr(self, "_f8", None)
        f8_fresh = f8 is not None and f8[0] == (self.weight.data_ptr(), self.weight._version)
        out = super()._apply(fn, *args, **kwargs)
        ver = (self.weight.data_ptr(), self.weight._version)
        if codes_fresh:
            self._codes_ver = ver
        if f8_fresh:
            dev = self.weight.device
            self._f8 = (ver, f8[1].to(dev), f8[2].to(dev))
        self._i8_sw = None
        return out

    # the fused-GEMM weight operand: (tensor, fmt, scales, group)
    def gemm_weight(self):
        """Integer codes while they still describe ``weight``; after a load_state_dict or an
        in-place edit of the buffer (data pointer / version changed) the codes are stale and
        dropped, and the GEMM runs on the fp16 buffer (the reference's own operand)."""
        if self.qcodes is not None:
            if getattr(self, "_codes_ver", None) == (self.weight.data_ptr(), self.weight._version):
                return self.qcodes, self.qfmt, self.qscales, self.qgroup
            self.drop_codes()
        return self.weight, "f16", None, 0

    def drop_codes(self):
        self.qcodes = None
        self.qscales = None
        self.qfmt = "f16"
        self.qgroup = 0
        self._codes_ver = None
        self.int8_mfma = False

    def i8_operand(self):
        """(int8 codes [N, K], fp32 scales [N]) of the int8-MFMA mode, or None when the layer is
        not in that mode (or its codes went stale)."""
        if not self.int8_mfma:
            return None
        w, fmt, sc, g = self.gemm_weight()
        if fmt != "i8" or g != self.in_features:
            return None
        cache = getattr(self, "_i8_sw", None)
        if cache is None or cache[0] != (sc.data_ptr(), sc._version):
            self._i8_sw = ((sc.data_ptr(), sc._version), sc.float().reshape(-1).contiguous())
        return w, self._i8_sw[1]

    def f8_operand(self):
        """(e4m3 weight bytes [N, K], fp32 group scales [K / 128, N]) of the W4A8-fp8 mode, or None
        (layer not in that mode, or its codes went stale)."""
        if not self.fp8_act:
            return None
        cache = getattr(self, "_f8", None)
        if cache is None or cache[0] != (self.weight.data_ptr(), self.weight._version):
            return None
        return cache[1], cache[2]

    def set_fp8(self, codes, scales, group, n_bits):
        """Build the fp8 operand from the W4 codes (exact in e4m3) and their group-128 scales."""
        if n_bits > 4 or group != 128 or self.in_features % 128 != 0 or self.out_features % 8 != 0:
            return False
        w8, gs = K.fp8_weight(codes.reshape(self.out_features, self.in_features).to(torch.int8),
                              scales.reshape(self.out_features, -1).to(torch.float16), group)
        self._f8 = ((self.weight.data_ptr(), self.weight._version), w8, gs)
        self.fp8_act = True
        return True

    def set_codes(self, codes, scales, group, n_bits):
        """Attach integer codes for the fused-dequant GEMM (int4 packed when n_bits <= 4)."""
        K_ = self.in_features
        if group % 32 != 0 or K_ % 64 != 0 or K_ % group != 0 or n_bits > 8:
            return False
        if n_bits <= 4:
            self.qcodes = K.pack_int4(codes.reshape(self.out_features, K_).contiguous())
            self.qfmt = "i4"
        else:
            self.qcodes = codes.reshape(self.out_features, K_).contiguous()
            self.qfmt = "i8"
        self.qscales = scales.reshape(self.out_features, K_ // group).contiguous()
        self.qgroup = group
        self.n_bits_W = n_bits
        self._codes_ver = (self.weight.data_ptr(), self.weight._version)
        return True

    @torch.no_grad()
    def forward(self, x):
        _need_gpu(x, "WxAxLinear")
        if x.dtype != torch.float16:
            raise RuntimeError(f"WxAxLinear expects fp16 input (the reference module's dtype), got {x.dtype}")
        q_x = self.act_quant(x) if self.quantize_act else x
        shape = q_x.shape
        x2 = q_x.reshape(-1, shape[-1])
        if x2.stride(-1) != 1 or x2.stride(0) % 8 != 0 or x2.data_ptr() % 16 != 0:
            x2 = x2.contiguous()
        i8 = self.i8_operand()
        if i8 is not None:
            xq, sa = K.quant_rows_i8(x2)
            y = K.linear_i8(xq, sa, i8[0], i8[1], bias=self.bias)
            y = y.reshape(*shape[:-1], self.out_features)
            return self.output_quant(y).to(x.dtype)
        f8 = self.f8_operand()
        if f8 is not None:
            xq, sa = K.quant_rows_fp8(x2)
            y = K.linear_fp8(xq, sa, f8[0], f8[1], bias=self.bias)
            y = y.reshape(*shape[:-1], self.out_features)
            return self.output_quant(y).to(x.dtype)
        w, fmt, sc, g = self.gemm_weight()
        y = K.linear(x2, w, fmt, sc, g, bias=self.bias)
        y = y.reshape(*shape[:-1], self.out_features)
        return self.output_quant(y).to(x.dtype)

    @classmethod
    def from_linear(cls, module, init_only=False, weight_quant="per_channel", act_quant="per_token",
                    quantize_output=False, n_bits_W=8, n_bits_A=16, group_size_W=0):
        assert isinstance(module, torch.nn.Linear)
        return cls(module.in_features, module.out_features, module.bias is not None, act_quant=act_quant,
                   quantize_output=quantize_output, n_bits_A=n_bits_A)

    @staticmethod
    @torch.no_grad()
    def from_float(module, init_only=False, weight_quant="per_channel", act_quant="per_token",
                   quantize_output=False, n_bits_W=8, n_bits_A=16, group_size_W=0, codeBookQuantInd=False,
                   debugPath=[], debug=False, int8_mfma=False, fp8_act=False):
        """fake_quant.py:234-258.  int8_mfma=True (this build's int8-MFMA W8A8 mode): per-row
        8-bit weight codes (weight_quant forced to per_channel) and per-token int8 activations.
        fp8_act=True (this build's W4A8-fp8 mode): the 4-bit group-128 codes also as e4m3 for
        the fp8 GEMM with per-token e4m3 activations (layers it does not fit keep A16)."""
        if int8_mfma:
            weight_quant, n_bits_W = "per_channel", 8
        assert isinstance(module, torch.nn.Linear)
        new = WxAxLinear(module.in_features, module.out_features, module.bias is not None,
                         weight_quant=weight_quant, act_quant=act_quant, quantize_output=quantize_output,
                         n_bits_A=n_bits_A)
        new.to(module.weight.device)
        if init_only:
            return new
        if codeBookQuantInd:
            raise NotImplementedError("codebook weight quantization (genCodeBook.py) is out of scope")
        w = module.weight.detach()
        if weight_quant == "per_channel":
            codes, scales, wdq, g = quantize_weight_absmax_codes(w, n_bits_W, 0)
        elif weight_quant == "per_tensor":
            wdq = quantize_weight_per_tensor_absmax(w.to(torch.float16), n_bits_W)
            codes = None
        elif weight_quant == "group":
            codes, scales, wdq, g = quantize_weight_absmax_codes(w, n_bits_W, group_size_W)
        else:
            raise ValueError(f"Invalid weight_quant: {weight_quant}")  # fake_quant.py:252-253
        new.weight.copy_(wdq)
        if codes is not None and n_bits_W <= 8:
            new.set_codes(codes, scales, g, n_bits_W)
            if fp8_act:
                new.set_fp8(codes, scales, g, n_bits_W)
        new.weight_quant_name = weight_quant
        if module.bias is not None:
            new.bias.copy_(module.bias.to(torch.float16))
        new.int8_mfma = bool(int8_mfma) and new.qfmt == "i8"
        return new

    def __repr__(self):
        return (f"WxAxLinear({self.in_features}, {self.out_features}, bias={self.bias is not None}, "
                f"weight_quant={self.weight_quant_name}, act_quant={self.act_quant_name}, "
                f"output_quant={self.output_quant_name})")


class WxAxConv2d(nn.Module):
    """Drop-in for nn.Conv2d with fake-quantized weight and optional input+output activation
    fake-quant (``quantise_act = quantize_output``, fake_quant.py:263-398).

    The GEMM operand is the fp16 dequantized weight re-laid out as [Co][kh][kw][Ci_pad] (cached,
    non-persistent): the reference's conv granularity (one scale per (Co, Ci, kh) row of kw
    weights) stores >= 1 fp16 scale per 3 weights, so codes + scales would not be smaller
    than the fp16 weight itself.
    """

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 bias=True, act_group_size=1, weight_quant="per_tensor", act_quant="per_token",
                 quantize_output=False, n_bits_A=16):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.stride = (stride, stride) if isinstance(stride, int) else tuple(stride)
        self.padding = (padding, padding) if isinstance(padding, int) else tuple(padding)
        self.dilation = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
        self.groups = groups
        self.a_gs = act_group_size
        self.quantise_act = quantize_output
        self.n_bits_A = n_bits_A
        assert self.in_channels % self.groups == 0
        wshape = (out_channels, in_channels // groups, *self.kernel_size)
        self.register_buffer("weight", torch.zeros(wshape, dtype=torch.float16))
        if bias:
            self.register_buffer("bias", torch.zeros(out_channels, dtype=torch.float16))
        else:
            self.register_buffer("bias", None)
        self.register_buffer("w_khwc", None, persistent=False)
        # int8-MFMA W8A8 mode: [Co][kh][kw][Ci_pad] int8 codes (one scale per output channel) and
        # per-sample int8 activations (qd_conv2d_i8); None = the reference's fake-quant path
        self.register_buffer("i8_w", None, persistent=False)
        self.register_buffer("i8_sw", None, persistent=False)
        self.weight_quant_name = weight_quant
        if act_quant not in ("per_token", "per_tensor", "per_channel", "per_group"):
            raise ValueError(f"Invalid act_quant: {act_quant}")  # fake_quant.py:316-317
        self.act_quant_name = act_quant
        self.act_quant = _act_quant_fn(act_quant, n_bits_A, self.a_gs)
        if quantize_output:
            self.output_quant_name = self.act_quant_name
            self.output_quant = self.act_quant
        else:
            self.output_quant_name = "None"
            self.output_quant = _identity

    @property
    def ci_pad(self):
        return (self.in_channels + 7) // 8 * 8

    def _apply(self, fn, *args, **kwargs):
        """Module.to / .cuda / .half: int8-mode codes that describe ``weight`` before the move are
        re-stamped after it (and their fp32 scales kept fp32) instead of going stale - a stale
        code set would drop the conv to an A16 fp16 conv, since set_int8 turned the fake-quant off."""
        i8_fresh = self.i8_w is not None and \
            getattr(self, "_i8_ver", None) == (self.weight.data_ptr(), self.weight._version)
        out = super()._apply(fn, *args, **kwargs)
        if i8_fresh:
            self.i8_sw = self.i8_sw.float()
            self._i8_ver = (self.weight.data_ptr(), self.weight._version)
        return out

    def gemm_weight(self):
        """[Co][kh][kw][Ci_pad] fp16 view of ``weight`` (rebuilt if the buffer changed)."""
        ver = (self.weight.data_ptr(), self.weight._version)
        if self.w_khwc is None or getattr(self, "_khwc_ver", None) != ver:
            _need_gpu(self.weight, "WxAxConv2d")
            self.w_khwc = K.conv_weight_khwc(self.weight.contiguous(), self.ci_pad)
            self._khwc_ver = ver
        return self.w_khwc

    def i8_operand(self):
        """(int8 codes [Co, kh, kw, Ci_pad], fp32 scales [Co]) of the int8-MFMA mode while they
        still describe ``weight``, else None."""
        if self.i8_w is None:
            return None
        if getattr(self, "_i8_ver", None) != (self.weight.data_ptr(), self.weight._version):
            # the buffer was edited / reloaded: back to the reference's fake-quant conv on it, with
            # the activation quant set_int8 switched off restored
            self.i8_w = self.i8_sw = None
            saved = getattr(self, "_fq_saved", None)
            if saved is not None:
                self.quantise_act, self.output_quant_name, self.output_quant = saved
            return None
        return self.i8_w, self.i8_sw

    @torch.no_grad()
    def set_int8(self, w_orig):
        """int8-MFMA mode: per-output-channel RTN codes of the ORIGINAL weight over (kh, kw, Ci)
        (the fake-quant recipe, fake_quant.py:44-46, at this granularity); ``weight`` becomes
        their dequantized value so state_dict / the NCHW reference path stay consistent."""
        co, ci, kh, kw = self.weight.shape
        cip = self.ci_pad
        if cip % 64 or co % 8 or self.groups != 1 or self.dilation != (1, 1):
            return False
        khwc = K.conv_weight_khwc(w_orig.detach().to(torch.float16).contiguous(), cip)
        codes, scales, wdq = K.weight_quant(khwc.view(co, -1), kh * kw * cip, 8)
        self.weight.copy_(wdq.view(co, kh, kw, cip)[..., :ci].permute(0, 3, 1, 2))
        self.i8_w = codes.view(co, kh, kw, cip).contiguous()
        self.i8_sw = scales.float().view(-1).contiguous()
        self._i8_ver = (self.weight.data_ptr(), self.weight._version)
        self._fq_saved = (self.quantise_act, self.output_quant_name, self.output_quant)
        self.quantise_act = False
        self.output_quant_name = "None"
        self.output_quant = _identity
        return True

    def _check_supported(self):
        if self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("grouped / dilated convolutions are not used by the SD UNets and "
                                      "have no kernel in this build")
        if self.stride[0] != self.stride[1] or self.padding[0] != self.padding[1]:
            raise NotImplementedError("anisotropic stride/padding not supported")

    @torch.no_grad()
    def forward(self, x):
        """NCHW in / NCHW out, as the reference module (fake_quant.py:333-341)."""
        _need_gpu(x, "WxAxConv2d")
        if x.dtype != torch.float16:
            raise RuntimeError(f"WxAxConv2d expects fp16 input, got {x.dtype}")
        self._check_supported()
        i8 = self.i8_operand()
        if i8 is not None:
            xq, sa = K.quant_samples_i8(K.nchw_to_nhwc(x.contiguous(), self.ci_pad))
            y = K.conv2d_i8(xq, sa, i8[0], i8[1], self.in_channels, self.stride[0], self.padding[0], bias=self.bias)
            return K.nhwc_to_nchw(y).to(x.dtype)
        q_x = self.act_quant(x) if self.quantise_act else x
        xh = K.nchw_to_nhwc(q_x.contiguous(), self.ci_pad)
        y = K.conv2d_nhwc(xh, self.gemm_weight(), self.in_channels, self.stride[0], self.padding[0],
                          bias=self.bias)
        yc = K.nhwc_to_nchw(y)
        return self.output_quant(yc).to(x.dtype)

    @classmethod
    @torch.no_grad()
    def from_float(cls, module, init_only=False, weight_quant="per_tensor", act_quant="per_tensor",
                   act_group_size=1, quantize_output=False, n_bits_W=8, n_bits_A=16, group_size_W=0,
                   codeBookQuantInd=False, debugPath=[], debug=False, int8_mfma=False):
        """fake_quant.py:343-382.  int8_mfma=True: the int8-MFMA W8A8 mode where the conv allows
        it (Ci_pad % 64 == 0, Co % 8 == 0; others keep the reference's fake-quant path)."""
        assert isinstance(module, torch.nn.Conv2d)
        new = cls(module.in_channels, module.out_channels, module.kernel_size, module.stride, module.padding,
                  module.dilation, module.groups, module.bias is not None, act_quant=act_quant,
                  quantize_output=quantize_output, n_bits_A=n_bits_A, act_group_size=act_group_size)
        new.to(module.weight.device)
        if init_only:
            return new
        if codeBookQuantInd:
            raise NotImplementedError("codebook weight quantization (genCodeBook.py) is out of scope")
        w = module.weight.detach()
        if weight_quant == "per_channel":
            wdq = quantize_weight_per_channel_absmax(w.to(torch.float16), n_bits_W)
        elif weight_quant == "per_tensor":
            wdq = quantize_weight_per_tensor_absmax(w.to(torch.float16), n_bits_W)
        elif weight_quant == "group":
            # the reference asserts w.dim() == 2 here for a 4-D conv weight (fake_quant.py:41)
            wdq = quantize_weight_absmax(w, n_bits_W, group_size_W)
        else:
            raise ValueError(f"Invalid weight_quant: {weight_quant}")
        new.weight.copy_(wdq)
        new.weight_quant_name = weight_quant
        new.n_bits_W = n_bits_W
        if module.bias is not None:
            new.bias.copy_(module.bias.to(torch.float16))
        if int8_mfma and n_bits_W == 8 and new.set_int8(w):
            new.weight_quant_name = "per_out_channel_int8"
        return new

    def __repr__(self):
        s = f"WxAxConv2d({self.in_channels}, {self.out_channels}, "
        s += f"kernel_size={self.kernel_size}, stride={self.stride}"
        if self.padding != (0, 0):
            s += f", padding={self.padding}"
        if self.dilation != (1, 1):
            s += f", dilation={self.dilation}"
        if self.groups != 1:
            s += f", groups={self.groups}"
        if self.bias is None:
            s += ", bias=False"
        s += f", weight_quant={self.weight_quant_name}"
        s += f", act_quant={self.act_quant_name}"
        s += f", output_quant={self.output_quant_name})"
        return s
