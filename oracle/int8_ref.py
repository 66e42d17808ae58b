"""CPU restatement of the int8-MFMA W8A8 mode (TEST INFRASTRUCTURE ONLY: tests/, smoke(),
bench.py's cpu_baseline may use it; the product never imports oracle/).

The mode (include/qdiff.h "int8-MFMA W8A8 mode") keeps the reference's RTN code
recipe - quantize/fake_quant.py:44-46 (s = half(half(max(amax, 1e-5)) / qmax)) and :72 / :117
(q = rint(half(x / s))) - but at granularities that factor out of an integer dot product:
  * linear weights per output row (quantize_weight_absmax with group = in_features, :21-84),
  * conv weights per output channel over (kh, kw, Ci),
  * linear activations per token (quantize_activation_per_token_absmax's codes, :108-118),
  * conv activations per sample (one scale per n over C, H, W).
The product is exact in integers; the output is y = half(((float32)acc * sa) * sw + bias) with
every operation rounded in float32 (the GPU epilogue's order), so the HIP kernels must match this
restatement BIT FOR BIT.
"""
import numpy as np
import torch

F16, F32 = np.float16, np.float32
_CLAMP = F16(1e-5)


def _scale(amax):
    """s = half(half(max(amax, 1e-5)) / 127) (fp16 value, returned as float32)."""
    a = np.maximum(np.asarray(amax, F32).astype(F16), _CLAMP)
    return (a.astype(F32) / F32(127)).astype(F16).astype(F32)


def _codes(x, s):
    t = (np.asarray(x, F16).astype(F32) / s).astype(F16)
    return np.rint(t.astype(F32)).astype(np.int8)


def quant_rows_i8(x):
    """x [M, K] fp16 -> (codes int8 [M, K], scales float32 [M]) - dynamic per token."""
    x = np.asarray(x, F16)
    s = _scale(np.abs(x.astype(F32)).max(axis=1))
    return _codes(x, s[:, None]), s


def quant_samples_i8(x):
    """x [N, ...] fp16 -> (codes int8, scales float32 [N]) - one scale per sample."""
    x = np.asarray(x, F16)
    n = x.shape[0]
    s = _scale(np.abs(x.reshape(n, -1).astype(F32)).max(axis=1))
    return _codes(x, s.reshape((n,) + (1,) * (x.ndim - 1))), s


def weight_rows_i8(w2d):
    """Per-output-row weight codes of w2d [N, K] (conv: [Co, kh*kw*Ci]) -> (codes, scales [N])."""
    return quant_rows_i8(w2d)


def weight_rows_dequant(w2d):
    """The fp16 weight buffer the int8-mode modules hold: half(rint(half(w / s)) * s) with the
    FLOAT rint (a small negative weight keeps its -0.0, as the reference's fake-quant ops give;
    the integer code cannot) = quantize_weight_absmax with one group per row (fake_quant.py:21-84)."""
    w = np.asarray(w2d, F16)
    s = _scale(np.abs(w.astype(F32)).max(axis=1))[:, None]
    t = (w.astype(F32) / s).astype(F16)
    return (np.rint(t.astype(F32)) * s).astype(F16)


def _epilogue(acc, sa_rows, sw, bias=None, residual=None):
    """acc int64 [M, N] (exact); sa_rows [M] float32; sw [N] float32."""
    v = acc.astype(F32) * sa_rows.astype(F32)[:, None]
    v = v * sw.astype(F32)[None, :]
    if bias is not None:
        v = v + np.asarray(bias, F16).astype(F32)[None, :]
    y = v.astype(F16)
    if residual is not None:
        y = (y.astype(F32) + np.asarray(residual, F16).astype(F32)).astype(F16)
    return y


def linear_i8(xq, sa, wq, sw, bias=None, residual=None):
    """xq [M, K] int8, sa [M], wq [N, K] int8, sw [N] -> y [M, N] fp16."""
    # float64 BLAS GEMM: exact integer sums (|acc| < 2^53), unlike numpy's slow int64 matmul
    acc = (torch.from_numpy(xq.astype(np.float64)) @ torch.from_numpy(wq.astype(np.float64)).T).numpy().astype(np.int64)
    return _epilogue(acc, np.asarray(sa, F32), np.asarray(sw, F32), bias, residual)


def conv2d_i8(xq, sa, wq, sw, bias=None, stride=1, pad=0, residual=None):
    """NCHW: xq [N, Ci, H, W] int8, sa [N] (per sample), wq [Co, Ci, kh, kw] int8, sw [Co]
    -> y [N, Co, Ho, Wo] fp16.  The integer sums are formed in float64 (exact: |acc| < 2^53)."""
    n, ci, h, w = xq.shape
    co, _, kh, kw = wq.shape
    ho, wo = (h + 2 * pad - kh) // stride + 1, (w + 2 * pad - kw) // stride + 1
    # im2col + float64 GEMM (BLAS): exact integer sums, far faster than a float64 conv
    cols = torch.nn.functional.unfold(torch.from_numpy(xq.astype(np.float64)), (kh, kw), padding=pad, stride=stride)
    wm = torch.from_numpy(wq.reshape(co, -1).astype(np.float64))
    acc = (wm @ cols).numpy().astype(np.int64)            # [n, co, ho*wo]
    rows = acc.transpose(0, 2, 1).reshape(-1, co)
    sa_rows = np.repeat(np.asarray(sa, F32), ho * wo)
    res = None if residual is None else np.asarray(residual, F16).transpose(0, 2, 3, 1).reshape(-1, co)
    y = _epilogue(rows, sa_rows, np.asarray(sw, F32), bias, res)
    return np.ascontiguousarray(y.reshape(n, ho, wo, co).transpose(0, 3, 1, 2))
