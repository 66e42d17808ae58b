"""CPU restatement of the W4A8-fp8 mode for SD3.5 (TEST INFRASTRUCTURE ONLY: tests/ may use it;
the product never imports oracle/).

The mode (include/qdiff.h "fp8 activations") keeps the reference's W4 group-128
weight codes and scales (quantize/fake_quant.py:21-84, the same buffers the fake-quant path
dequantizes) and replaces the fp16 activation with per-token OCP e4m3 codes:
  s_m = max(amax_m, 1e-5) / 448 (f32),  x8 = e4m3(x / s_m) (round to nearest even, torch's
  float8_e4m3fn conversion), y = half(s_m * sum_g gs[g][n] * (x8 . q)_g + bias).
Codes and scales are bit-exact targets; the GEMM output is compared within the fp32 summation
bound (its sum is formed in float64 here).
"""
import torch

F16, F8 = torch.float16, torch.float8_e4m3fn


def quant_rows_fp8(x):
    """x fp16 [M, K] -> (e4m3 codes as uint8 [M, K], scales f32 [M])."""
    xf = x.float()
    s = xf.abs().amax(dim=1).clamp(min=1e-5) / 448.0
    q = (xf / s[:, None]).to(F8)
    return q.view(torch.uint8), s


def weight_codes(w, n_bits, group):
    """The reference's group RTN codes (quantize_weight_absmax, fake_quant.py:21-84, as
    oracle/fake_quant_torch.weight_group computes them): (codes int8 [N, K], scales fp16 [N, K/g])."""
    from .fake_quant_torch import _scale
    n, k = w.shape
    w2 = w.to(F16).reshape(-1, group)
    s = _scale(w2.abs().max(dim=-1, keepdim=True)[0], n_bits)
    q = w2.div(s).round()
    return q.to(torch.int8).reshape(n, k), s.reshape(n, k // group)


def decode(q8):
    return q8.view(F8).float()


def linear_fp8(xq, sa, codes, scales, group, bias=None):
    """Exact group sums in float64 -> (value before rounding f64 [M, N], y fp16, the |terms| sum
    for the accumulation-order bound)."""
    x = decode(xq).double()
    q = codes.double()
    m, k = x.shape
    n = q.shape[0]
    ng = k // group
    acc = torch.zeros(m, n, dtype=torch.float64)
    mag = torch.zeros(m, n, dtype=torch.float64)
    for g in range(ng):
        sl = slice(g * group, (g + 1) * group)
        part = x[:, sl] @ q[:, sl].t()
        sg = scales[:, g].double()[None, :]
        acc += part * sg
        mag += (x[:, sl].abs() @ q[:, sl].abs().t()) * sg.abs()
    v = acc * sa.double()[:, None]
    mag = mag * sa.double()[:, None]
    if bias is not None:
        v = v + bias.double()[None, :]
    return v, v.to(F16), mag
