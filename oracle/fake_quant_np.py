"""numpy restatement of the reference fake-quant operators (TEST INFRASTRUCTURE ONLY).

Every function follows /root/reference/quantize/fake_quant.py line by line in *semantics*
(SURVEY.md Appendix A): tensors are IEEE fp16, each elementwise op is computed in fp32 and
rounded to fp16 once (PyTorch CPU Half semantics; numpy's float16 ufuncs do the same),
``round_`` is round-half-to-even (``np.rint``), and ``clamp_(min=1e-5)`` on an fp16 tensor is
``max(x, half(1e-5))`` because no fp16 value lies strictly between 1e-5 and half(1e-5).

Pinned bit-exactly against tests/golden/fake_quant_golden.npz (generated from the reference's
own module by tests/golden/make_golden.py).
"""
import numpy as np

F16 = np.float16
_CLAMP = F16(1e-5)


def _qmax(n_bits):
    return 2 ** (n_bits - 1) - 1


def _scale_from_amax(amax, n_bits):
    # scales.clamp_(min=1e-5).div_(q_max)   fake_quant.py:45-46, 114-116, 127-129
    amax = np.maximum(amax.astype(F16), _CLAMP)
    return (amax.astype(np.float32) / np.float32(_qmax(n_bits))).astype(F16)


def _qdq(x, s):
    # t.div_(scales).round_().mul_(scales)   fake_quant.py:72, 92, 104, 117, 130
    t = (x.astype(np.float32) / s.astype(np.float32)).astype(F16)
    q = np.rint(t)
    return (q.astype(np.float32) * s.astype(np.float32)).astype(F16)


def shrink_group(k, group_size, step=32):
    """Group-size shrink rule of fake_quant.py:33-37 (``while K % g: g -= 32``).

    The reference loops until ``K % g == 0``; a g that reaches 0 raises ZeroDivisionError
    there (``K % 0``), which we reproduce.
    """
    g = group_size
    while k % g != 0:
        g -= step
        if g == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
    return g


def quantize_weight_absmax(w, n_bits=8, group_size=0):
    """fake_quant.py:21-84 (codebook branch off).  Group absmax RTN, groups along the last dim."""
    w = np.asarray(w, dtype=F16)
    shape = w.shape
    if group_size > 0:
        g = shrink_group(shape[-1], group_size)
        w2 = w.reshape(-1, g)
    else:
        w2 = w
    if w2.ndim != 2:
        raise AssertionError("w.dim() == 2")          # fake_quant.py:41
    if np.isnan(w2).any():
        raise AssertionError("NaN in weight")          # fake_quant.py:42
    s = _scale_from_amax(np.abs(w2).max(axis=-1, keepdims=True), n_bits)
    out = _qdq(w2, s)
    return out.reshape(shape).astype(F16)


def quantize_weight_absmax_codes(w, n_bits=8, group_size=0):
    """Integer codes + fp16 scales such that ``half(codes * scales)`` equals
    :func:`quantize_weight_absmax` (the on-device storage format of the product path)."""
    w = np.asarray(w, dtype=F16)
    shape = w.shape
    g = shrink_group(shape[-1], group_size) if group_size > 0 else shape[-1]
    w2 = w.reshape(-1, g)
    s = _scale_from_amax(np.abs(w2).max(axis=-1, keepdims=True), n_bits)
    t = (w2.astype(np.float32) / s.astype(np.float32)).astype(F16)
    q = np.rint(t).astype(np.int8)
    return q.reshape(shape), s.reshape(shape[:-1] + (shape[-1] // g,)), g


def quantize_weight_per_channel_absmax(w, n_bits=8):
    """fake_quant.py:86-93: absmax over the LAST dim (for a 4-D conv weight: per (Co,Ci,kh))."""
    w = np.asarray(w, dtype=F16)
    s = _scale_from_amax(np.abs(w).max(axis=-1, keepdims=True), n_bits)
    return _qdq(w, s)


def quantize_weight_per_tensor_absmax(w, n_bits=8):
    """fake_quant.py:96-105."""
    w = np.asarray(w, dtype=F16)
    s = _scale_from_amax(np.abs(w).max(), n_bits)
    return _qdq(w, s)


def quantize_activation_per_token_absmax(t, n_bits=8):
    """fake_quant.py:108-118: one scale per row of ``t.view(-1, C)``."""
    t = np.asarray(t, dtype=F16)
    t2 = t.reshape(-1, t.shape[-1])
    s = _scale_from_amax(np.abs(t2).max(axis=-1, keepdims=True), n_bits)
    return _qdq(t2, s).reshape(t.shape)


def quantize_activation_per_channel_absmax(t, n_bits=8):
    """fake_quant.py:123-131: NCHW, one scale per (n, c) over (H, W)."""
    t = np.asarray(t, dtype=F16)
    s = _scale_from_amax(np.abs(t).max(axis=(2, 3), keepdims=True), n_bits)
    return _qdq(t, s)


def per_group_size(h, w, group_size):
    """fake_quant.py:138-139: ``while H % g or W % g: g -= 2``."""
    g = group_size
    while h % g != 0 or w % g != 0:
        g -= 2
        if g == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
    return g


def quantize_activation_per_channel_group_absmax(t, group_size=128, n_bits=8):
    """fake_quant.py:133-153: one scale per (n, c, g×g spatial patch)."""
    t = np.asarray(t, dtype=F16)
    n, c, h, w = t.shape
    g = per_group_size(h, w, group_size)
    p = t.reshape(n, c, h // g, g, w // g, g)
    s = _scale_from_amax(np.abs(p).max(axis=(3, 5), keepdims=True), n_bits)
    return _qdq(p, s).reshape(n, c, h, w)


def quantize_activation_per_tensor_absmax(t, n_bits=8):
    """fake_quant.py:157-167."""
    t = np.asarray(t, dtype=F16)
    s = _scale_from_amax(np.abs(t).max(), n_bits)
    return _qdq(t, s)


def pseudo_quantize_tensor(w, n_bits=4, group_size=128, zero_point=True):
    """AwqQuantizer.pseudo_quantize_tensor (quantizer.py:163-198), fp16 op-by-op.

    Not on the diffusion path; kept for completeness of the
    quantizer surface.  Returns (w_dq, scales, zeros-or-None).
    """
    w = np.asarray(w, dtype=F16)
    shape = w.shape
    if group_size > 0:
        assert shape[-1] % group_size == 0
        w = w.reshape(-1, group_size)
    f32 = np.float32
    if zero_point:
        mx = w.max(axis=1, keepdims=True)
        mn = w.min(axis=1, keepdims=True)
        max_int = 2 ** n_bits - 1
        rng = (mx.astype(f32) - mn.astype(f32)).astype(F16)
        rng = np.maximum(rng, _CLAMP)
        s = (rng.astype(f32) / f32(max_int)).astype(F16)
        z = np.rint((mn.astype(f32) / s.astype(f32)).astype(F16))
        z = np.clip((-z).astype(F16), 0, max_int).astype(F16)
        t = np.rint((w.astype(f32) / s.astype(f32)).astype(F16))
        t = (t.astype(f32) + z.astype(f32)).astype(F16)
        t = np.clip(t, 0, max_int).astype(F16)
        t = (t.astype(f32) - z.astype(f32)).astype(F16)
        out = (t.astype(f32) * s.astype(f32)).astype(F16)
        zeros = z.reshape(shape[0], -1)
    else:
        mx = np.maximum(np.abs(w).max(axis=1, keepdims=True), _CLAMP)
        max_int = 2 ** (n_bits - 1) - 1
        min_int = -(2 ** (n_bits - 1))
        s = (mx.astype(f32) / f32(max_int)).astype(F16)
        t = np.rint((w.astype(f32) / s.astype(f32)).astype(F16))
        t = np.clip(t, min_int, max_int).astype(F16)
        out = (t.astype(f32) * s.astype(f32)).astype(F16)
        zeros = None
    return out.reshape(shape), s.reshape(shape[0], -1), zeros


def smooth_scales(act_absmax, fc_weights, alpha=0.8):
    """SqQuantizer.smooth_ln_fcs scale (quantizer_SQ.py:416-424), fp16 op-by-op.

    weight_scales = max over fcs of |W|.max(dim=0), clamp 1e-5;
    scales = clamp(act**alpha / weight_scales**(1-alpha), 1e-5).
    torch's Half ``pow(Scalar)`` first rounds the exponent to the tensor dtype (measured against
    the reference in make_golden: pow(x, 0.8) == half(float(x) ** float(half(0.8)))).
    """
    f32 = np.float32
    ws = np.stack([np.abs(np.asarray(w, F16)).max(axis=0) for w in fc_weights]).max(axis=0)
    ws = np.maximum(ws, _CLAMP)
    a = np.asarray(act_absmax, F16)
    ea = np.float64(F16(alpha))
    eb = np.float64(F16(1 - alpha))
    num = np.power(a.astype(np.float64), ea).astype(f32).astype(F16)
    den = np.power(ws.astype(np.float64), eb).astype(f32).astype(F16)
    s = (num.astype(f32) / den.astype(f32)).astype(F16)
    return np.maximum(s, _CLAMP)
