"""AWQ activation-aware scale search and weight-clip search for the UNet's transformer blocks
(quantize(..., quantType="awq", awq_search=True)).

The reference implements both searches for LLMs (quantize/quantizer.py:604-720
``_search_best_scale`` / ``_compute_best_scale``, :799-863 ``_search_best_clip`` /
``_compute_best_clip``) and switches them off for diffusion models (``calibrate = False``,
quantizer.py:1050: the diffusion branch is plain RTN).  This module runs them for the UNet on
device, with the groupings the SmoothQuant adapter already defines for the blocks
(StableDiffusion1_x.py:115-150: norm1 -> attn1.to_q / to_k / to_v, norm3 -> ff.net.0.proj; plus
norm2 -> attn2.to_q, the only cross-attention projection fed by a norm) and the diffusion
branch's own weight quantizer as Q (quantize_weight_absmax, fake_quant.py:21-84, the one the
final swap applies) instead of the LLM path's zero-point pseudo_quantize_tensor.

Per group, with X the block input captured during a calibration run (a strided row sample per
forward call):
  scale search   s(r) = (mean|X|^r / (w_mean^(1-r) + 1e-4)).clamp(1e-4) / sqrt(max * min),
                 r = 0, 1/20, ..., 19/20;  loss(r) = mean (X W^T - X (Q(W s) / s)^T)^2 over every
                 layer of the group; the best s is folded as the reference's apply_scale does for a
                 LayerNorm prev-op: ln.weight /= s, ln.bias /= s, W *= s.
  clip search    per linear (names containing "q_", "k_", "query", "key" or "Wqkv" skipped, the
                 reference's avoid list), per (output channel, weight group): max_val =
                 amax * (1 - i/20), i < 10, minimizing mean over sampled tokens of the group's
                 partial output error; the weight is clamped to +-max_val (apply_clip).
GEMMs run on libqdiff (qd_linear_fwd), the weight fake-quant on qd_weight_quant; the per-channel
statistics and loss reductions are small device tensor ops at quantize time.
"""
import torch
from torch import nn

from . import kernels as K
from .fake_quant import quantize_weight_absmax, shrink_group

N_GRID = 20
MAX_SHRINK = 0.5
N_SAMPLE_TOKEN = 512
# quantizer.py:788-791 skips the q / k projections ("due to qk bmm, it is hard to clip precisely")
# by LLM substrings; diffusers names them attn*.to_q / to_k (UNet) and add_q_proj / add_k_proj
# (MMDiT), matched on the final name component
AVOID_CLIP = ("q_", "k_", "query", "key", "Wqkv")
AVOID_CLIP_LEAF = ("to_q", "to_k", "add_q_proj", "add_k_proj")


def clip_avoided(lname):
    leaf = lname.split(".")[-1]
    return any(a in lname for a in AVOID_CLIP) or leaf in AVOID_CLIP_LEAF


class InputCapture:
    """A linear's input rows during calibration: `per_call` rows strided over each call's
    tokens, up to `max_rows` in total (spread over every denoising step of the run)."""

    def __init__(self, per_call=8, max_rows=4096):
        self.per_call, self.max_rows = per_call, max_rows
        self.chunks, self.rows = [], 0

    def __call__(self, x2d):
        if self.rows >= self.max_rows:
            return
        step = max(1, x2d.shape[0] // self.per_call)
        xs = x2d[::step][: self.per_call].clone()
        self.chunks.append(xs)
        self.rows += xs.shape[0]

    def data(self):
        if not self.chunks:
            raise RuntimeError("AWQ search: a linear recorded no calibration input")
        return torch.cat(self.chunks).contiguous()


def _linear_out(x, w, bias):
    return K.linear(x, w.contiguous(), "f16", bias=None if bias is None else bias.detach().contiguous())


def _mse(a, b):
    return float((a.float() - b.float()).pow(2).mean())


def _q(w, n_bits, group):
    return quantize_weight_absmax(w, n_bits, group)


@torch.no_grad()
def search_scale(x, layers, n_bits, group_size):
    """_compute_best_scale on device -> (best scales fp16 [C], best ratio, {ratio: loss})."""
    w = torch.cat([l.weight.detach() for l in layers], 0)
    g = shrink_group(w.shape[1], group_size) if group_size > 0 else w.shape[1]
    wg = w.float().view(-1, g)
    w_scale = (wg.abs() / (wg.abs().amax(dim=1, keepdim=True) + 1e-6)).view(w.shape)
    w_mean = w_scale.mean(0)
    x_mean = x.float().abs().mean(0)
    ref = [_linear_out(x, l.weight.detach(), l.bias) for l in layers]
    history, best = {}, (float("inf"), None, None)
    for i in range(N_GRID):
        r = i / N_GRID
        s = (x_mean.pow(r) / (w_mean.pow(1 - r) + 1e-4)).clamp(min=1e-4)
        s = s / (s.max() * s.min()).sqrt()
        s[torch.isinf(s) | torch.isnan(s)] = 1
        s16 = s.to(torch.float16)
        loss = 0.0
        for l, y0 in zip(layers, ref):
            wq = (_q((l.weight.detach() * s16).contiguous(), n_bits, group_size) / s16).contiguous()
            loss += _mse(y0, _linear_out(x, wq, l.bias)) * y0.numel()
        loss /= sum(y.numel() for y in ref)
        history[r] = loss
        if loss < best[0]:
            best = (loss, r, s16.clone())
    if best[1] is None:
        raise RuntimeError(f"AWQ scale search found no finite loss: {history}")
    return best[2], best[1], history


@torch.no_grad()
def apply_scale_ln(ln, layers, s):
    """apply_scale for a LayerNorm prev-op (fp16 in-place ops): ln.w /= s, ln.b /= s, W *= s."""
    ln.weight.div_(s)
    if ln.bias is not None:
        ln.bias.div_(s)
    for l in layers:
        l.weight.mul_(s.view(1, -1))


@torch.no_grad()
def search_clip(w, x, n_bits, group_size):
    """_compute_best_clip on device -> best max_val [co, n_group] fp16."""
    co, ci = w.shape
    g = shrink_group(ci, group_size) if group_size > 0 else ci
    ng = ci // g
    step = max(1, x.shape[0] // N_SAMPLE_TOKEN)
    xs = x[::step].contiguous()
    wf = w.detach()
    org_max = wf.abs().view(co, ng, g).amax(dim=-1)                   # [co, ng]
    xg = [xs[:, j * g:(j + 1) * g].contiguous() for j in range(ng)]
    org = [_linear_out(xg[j], wf[:, j * g:(j + 1) * g], None) for j in range(ng)]
    best = org_max.clone()
    min_err = torch.full((co, ng), float("inf"), device=w.device)
    for i in range(int(MAX_SHRINK * N_GRID)):
        mv = org_max * (1 - i / N_GRID)
        mvx = mv.repeat_interleave(g, dim=1)
        cur = torch.maximum(torch.minimum(wf, mvx), -mvx)
        qw = _q(cur.contiguous(), n_bits, group_size)
        for j in range(ng):
            out = _linear_out(xg[j], qw[:, j * g:(j + 1) * g], None)
            err = (out.float() - org[j].float()).pow(2).mean(0)    # [co]
            better = err < min_err[:, j]
            min_err[better, j] = err[better]
            best[better, j] = mv[better, j]
    return best


@torch.no_grad()
def apply_clip(layer, max_val):
    co, ci = layer.weight.shape
    ng = max_val.shape[1]
    mvx = max_val.repeat_interleave(ci // ng, dim=1).to(layer.weight.dtype)
    layer.weight.data = torch.maximum(torch.minimum(layer.weight.data, mvx), -mvx).contiguous()


def scale_groups(block):
    """(prev LayerNorm, linears fed by it) of one BasicTransformerBlock."""
    return [(block.norm1, [block.attn1.to_q, block.attn1.to_k, block.attn1.to_v]),
            (block.norm2, [block.attn2.to_q]),
            (block.norm3, [block.ff.net[0].proj])]


@torch.no_grad()
def run_awq_search(adapter, n_bits, group_size, calibration=None, clip=True):
    """Calibrate with input captures on every linear of every transformer block, then scale
    search + fold per group, then clip search per eligible linear.  Returns a report dict."""
    blocks = adapter.get_smoothing_blocks()
    caps = {}
    for bname, blk in blocks.items():
        for lname, sub in blk.named_modules():
            if isinstance(sub, nn.Linear):
                cap = InputCapture()
                sub._qd_hook = cap
                caps[(bname, lname)] = (sub, cap)
    try:
        adapter.run_sq_calibration(**(calibration or {}))
    finally:
        for sub, _ in caps.values():
            if hasattr(sub, "_qd_hook"):
                del sub._qd_hook
    report = {"scales": {}, "clips": 0}
    folded = {}   # id(linear) -> the scale folded into its input LayerNorm
    for bname, blk in blocks.items():
        names = {id(m): n for n, m in blk.named_modules()}
        for ln, layers in scale_groups(blk):
            x = caps[(bname, names[id(layers[0])])][1].data()
            s, r, hist = search_scale(x, layers, n_bits, group_size)
            apply_scale_ln(ln, layers, s)
            for l in layers:
                folded[id(l)] = s
            report["scales"][f"{bname}.{names[id(ln)]}"] = {"ratio": r, "loss": hist[r], "loss_ratio0": hist[0.0]}
    if clip:
        for (bname, lname), (sub, cap) in caps.items():
            if clip_avoided(lname):
                continue
            x = cap.data()
            if id(sub) in folded:   # the fold divided this layer's input by s (and scaled W by s)
                x = (x / folded[id(sub)]).to(x.dtype).contiguous()
            apply_clip(sub, search_clip(sub.weight, x, n_bits, group_size))
            report["clips"] += 1
    return report


__all__ = ["run_awq_search", "search_scale", "search_clip", "apply_scale_ln", "apply_clip", "InputCapture",
           "scale_groups", "N_GRID", "AVOID_CLIP", "clip_avoided"]
