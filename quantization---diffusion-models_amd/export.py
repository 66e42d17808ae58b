"""On-disk integer formats of the quantized layers.

* AWQ GEMM int4 layout (the format AutoAWQ's WQLinear_GEMM kernels and the reference's own
  utilities read, utils/quant_utils.py:14-67 pack/unpack, utils/packing_utils.py:4-40 AWQ_ORDER
  [0, 2, 4, 6, 1, 3, 5, 7] / unpack_awq / reverse_awq_order / dequantize_gemm): per linear
  ``qweight`` int32 [in_features, out_features / 8] (eight 4-bit codes along the output dim, nibble
  i holding column 8c + AWQ_ORDER[i]), ``qzeros`` int32 [in / group, out / 8] (same packing),
  ``scales`` fp16 [in / group, out].  This build's symmetric RTN codes q in [-8, 7]
  (fake_quant.py:21-84) are stored as u = q + 8 with zero point 8, so the reference's
  dequantize_gemm ((u - z) * s) reproduces the WxAxLinear weight buffer bit for bit.
* Conv codes: the reference's per-(Co, Ci, kh) conv granularity (fake_quant.py:86-93) as int8
  codes [Co, Ci, kh, kw] + fp16 scales [Co, Ci, kh]; the int8-MFMA mode's per-output-channel
  codes [Co, kh, kw, Ci_pad] + fp32 scales.
Format conversion only (offline, host / torch ops): never on the denoising path.
"""
import torch

AWQ_ORDER = (0, 2, 4, 6, 1, 3, 5, 7)


def _pack_cols(u):
    """[R, C] values in [0, 15] -> int32 [R, C / 8], nibble i of word c = column 8c + AWQ_ORDER[i]."""
    r, c = u.shape
    if c % 8:
        raise ValueError("AWQ packing needs a multiple of 8 columns")
    v = u.to(torch.int64).view(r, c // 8, 8)[:, :, list(AWQ_ORDER)]
    shifts = torch.arange(0, 32, 4, device=u.device, dtype=torch.int64)
    word = (v << shifts).sum(-1)
    return torch.where(word >= 2 ** 31, word - 2 ** 32, word).to(torch.int32)


def _unpack_cols(q):
    """Inverse of _pack_cols: int32 [R, C / 8] -> int8 [R, C] in [0, 15]."""
    r, c8 = q.shape
    shifts = torch.arange(0, 32, 4, device=q.device, dtype=torch.int64)
    v = ((q.to(torch.int64) & 0xFFFFFFFF)[:, :, None] >> shifts) & 0xF
    inv = [AWQ_ORDER.index(i) for i in range(8)]
    return v[:, :, inv].reshape(r, c8 * 8).to(torch.int8)


def awq_pack_linear(codes, scales, group):
    """Symmetric int4 codes [N, K] (int8 storage, values in [-8, 7]) + scales [N, K / g] ->
    dict(qweight int32 [K, N / 8], qzeros int32 [K / g, N / 8], scales fp16 [K / g, N])."""
    n, k = codes.shape
    if k % group or scales.shape != (n, k // group):
        raise ValueError("codes / scales / group mismatch")
    if int(codes.min()) < -8 or int(codes.max()) > 7:
        raise ValueError("AWQ int4 export needs codes in [-8, 7] (w_bit <= 4)")
    u = (codes.to(torch.int16) + 8).t().contiguous()
    z = torch.full((k // group, n), 8, dtype=torch.int16, device=codes.device)
    return {"qweight": _pack_cols(u), "qzeros": _pack_cols(z), "scales": scales.t().contiguous().to(torch.float16)}


def awq_unpack_linear(qweight, qzeros, scales, group):
    """AWQ GEMM tensors -> (codes int8 [N, K] in [-8, 7], scales fp16 [N, K / g]); raises unless
    every zero point is 8 (this build's symmetric codes)."""
    u = _unpack_cols(qweight)
    z = _unpack_cols(qzeros)
    if not bool((z == 8).all()):
        raise ValueError("asymmetric AWQ zero points: not this build's symmetric RTN codes")
    return (u.to(torch.int16) - 8).to(torch.int8).t().contiguous(), scales.t().contiguous()


def packed_nibbles_to_codes(packed, k):
    """This build's GEMM layout -> int8 [N, K]: per 8-code word (one little-endian dword, k = 8i ..
    8i + 7) nibble j holds q(8i + 2j) + 8 and nibble j + 4 holds q(8i + 2j + 1) + 8 (qd_pack_int4)."""
    n = packed.shape[0]
    w = packed.contiguous().view(torch.uint8).reshape(n, -1, 4).to(torch.int32)
    w = w[..., 0] | (w[..., 1] << 8) | (w[..., 2] << 16) | (w[..., 3] << 24)
    shifts = torch.tensor([0, 16, 4, 20, 8, 24, 12, 28], dtype=torch.int32, device=packed.device)
    c = (w[..., None] >> shifts) & 0xF
    return (c - 8).to(torch.int8).reshape(n, k)


@torch.no_grad()
def conv_codes(weight, n_bits):
    """The reference's conv weight quant (per (Co, Ci, kh) row of kw values, fake_quant.py:86-93)
    as integer codes: (codes int8 [Co, Ci, kh, kw], scales fp16 [Co, Ci, kh])."""
    from . import kernels as K
    co, ci, kh, kw = weight.shape
    codes, scales, _ = K.weight_quant(weight.reshape(-1, kw).contiguous(), kw, n_bits, want_dq=False)
    return codes.view(co, ci, kh, kw), scales.view(co, ci, kh)


def dequant_conv_codes(codes, scales):
    """half(q * s) with the per-(Co, Ci, kh) scale (exact: |q| <= 127, s fp16)."""
    return (codes.float() * scales.float()[..., None]).to(torch.float16)
