"""torch-CPU restatement of the reference fake-quant math (TEST INFRASTRUCTURE / CPU BASELINE).

Same semantics as oracle/fake_quant_np.py (Appendix A of SURVEY.md), written with torch CPU
fp16 ops - which is what the reference itself executes (quantize/fake_quant.py:21-167 run on
CPU Half tensors).  Used by the CPU UNet oracle (oracle/unet_ref.py) for speed; pinned by
the same golden fixtures as the numpy version (tests/test_oracle_golden.py).
"""
import torch

_CLAMP = 1e-5


def _qdq(x, s):
    return x.div(s).round_().mul_(s)


def _scale(amax, n_bits):
    return amax.clamp_(min=_CLAMP).div_(2 ** (n_bits - 1) - 1)


@torch.no_grad()
def per_token(t, n_bits=8):
    """fake_quant.py:108-118."""
    shape = t.shape
    t2 = t.contiguous().view(-1, shape[-1])
    s = _scale(t2.abs().max(dim=-1, keepdim=True)[0], n_bits)
    return _qdq(t2, s).view(shape)


@torch.no_grad()
def per_channel(t, n_bits=8):
    """fake_quant.py:123-131 (NCHW)."""
    s = _scale(torch.amax(t.abs(), dim=(2, 3), keepdim=True), n_bits)
    return _qdq(t, s)


@torch.no_grad()
def per_tensor(t, n_bits=8):
    """fake_quant.py:157-167."""
    s = _scale(t.abs().max(), n_bits)
    return _qdq(t, s)


@torch.no_grad()
def per_group(t, group_size=128, n_bits=8):
    """fake_quant.py:133-153."""
    n, c, h, w = t.shape
    g = group_size
    while h % g != 0 or w % g != 0:
        g -= 2
        if g == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
    p = t.unfold(2, g, g).unfold(3, g, g)
    s = _scale(torch.amax(p.abs(), dim=(4, 5), keepdim=True), n_bits)
    q = p.div(s).round().mul(s)
    return q.permute(0, 1, 2, 4, 3, 5).contiguous().view(n, c, h, w)


ACT = {"per_token": per_token, "per_channel": per_channel, "per_tensor": per_tensor}


def _shrink(k, g):
    while k % g != 0:
        g -= 32
        if g == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
    return g


@torch.no_grad()
def weight_group(w, n_bits=8, group_size=0):
    """quantize_weight_absmax (fake_quant.py:21-84) on a CPU fp16 tensor (not in place)."""
    shape = w.shape
    w2 = w.clone()
    if group_size > 0:
        w2 = w2.reshape(-1, _shrink(shape[-1], group_size))
    assert w2.dim() == 2
    s = _scale(w2.abs().max(dim=-1, keepdim=True)[0], n_bits)
    return _qdq(w2, s).reshape(shape)


@torch.no_grad()
def weight_per_channel(w, n_bits=8):
    """fake_quant.py:86-93."""
    s = _scale(w.abs().max(dim=-1, keepdim=True)[0], n_bits)
    return _qdq(w, s)


@torch.no_grad()
def weight_per_tensor(w, n_bits=8):
    """fake_quant.py:96-105."""
    s = _scale(w.abs().max(), n_bits)
    return _qdq(w, s)
