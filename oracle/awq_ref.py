"""CPU restatement of the AWQ scale / clip searches run on the UNet (awq_search.py) - TEST
INFRASTRUCTURE ONLY (tests/ use it; the product never imports oracle/).

Follows the reference's LLM searches (quantize/quantizer.py:667-720 _compute_best_scale and
:822-863 _compute_best_clip) with Q = the diffusion branch's group RTN weight fake-quant
(oracle/fake_quant_torch.weight_group, pinned bit-exact to the reference's goldens), GEMMs in
fp32 rounded to fp16 once (the GPU path's arithmetic).  Parity of the search itself is unpinned
(the reference never runs it for diffusion models): these functions restate its published
algorithm so the GPU search can be checked against the same loss landscape.
"""
import torch

from . import fake_quant_torch as FT

F16 = torch.float16
N_GRID = 20


def _group(k, group_size):
    g = group_size
    while k % g:
        g -= 32
    return g


def _lin(x, w, b=None):
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    return y.half()


def scale_losses(x, ws, bs, n_bits, group_size):
    """{ratio: loss} and the scales per ratio of _compute_best_scale (duo_scaling)."""
    w = torch.cat(ws, 0)
    g = _group(w.shape[1], group_size)
    wg = w.float().view(-1, g)
    w_mean = (wg.abs() / (wg.abs().amax(dim=1, keepdim=True) + 1e-6)).view(w.shape).mean(0)
    x_mean = x.float().abs().mean(0)
    ref = [_lin(x, wi, bi) for wi, bi in zip(ws, bs)]
    out, scales = {}, {}
    for i in range(N_GRID):
        r = i / N_GRID
        s = (x_mean.pow(r) / (w_mean.pow(1 - r) + 1e-4)).clamp(min=1e-4)
        s = s / (s.max() * s.min()).sqrt()
        s[torch.isinf(s) | torch.isnan(s)] = 1
        s16 = s.half()
        tot, n = 0.0, 0
        for wi, bi, y0 in zip(ws, bs, ref):
            wq = FT.weight_group((wi * s16).contiguous(), n_bits, group_size) / s16
            d = (_lin(x, wq, bi).float() - y0.float()).pow(2)
            tot += float(d.sum())
            n += d.numel()
        out[r] = tot / n
        scales[r] = s16
    return out, scales


def clip_errors(w, x, max_vals, n_bits, group_size):
    """Mean squared partial-output error per (output channel, group) of the weight clamped to
    +-max_vals [co, n_group] and fake-quantized (the quantity _compute_best_clip minimizes)."""
    co, ci = w.shape
    g = _group(ci, group_size)
    ng = ci // g
    step = max(1, x.shape[0] // 512)
    xs = x[::step]
    mvx = max_vals.float().repeat_interleave(g, dim=1).half()
    cur = torch.maximum(torch.minimum(w, mvx), -mvx)
    qw = FT.weight_group(cur.contiguous(), n_bits, group_size)
    err = torch.empty(co, ng)
    for j in range(ng):
        sl = slice(j * g, (j + 1) * g)
        o = _lin(xs[:, sl], qw[:, sl]).float()
        o0 = _lin(xs[:, sl], w[:, sl]).float()
        err[:, j] = (o - o0).pow(2).mean(0)
    return err
