"""Host checks of oracle/fused_ref.py, the per-launch restatement test_gpu_c2.py uses: its fused
compositions equal the unfused reference ops they stand for (fake_quant_torch, torch-CPU)."""
import torch
import torch.nn.functional as F

from oracle import fake_quant_torch as FT
from oracle import fused_ref as FR


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).half()


def test_finalize_is_per_channel_fake_quant_plus_residual():
    y = _r(2, 4, 4, 16, seed=1, scale=3)
    res = _r(2, 4, 4, 16, seed=2)
    amax = y.float().abs().reshape(2, -1, 16).amax(1)
    got = FR.finalize(y, amax, 8, residual=res)
    ref = FT.per_channel(y.permute(0, 3, 1, 2).contiguous(), 8).permute(0, 2, 3, 1)
    ref = (ref.float() + res.float()).half()
    assert torch.equal(got, ref)
    cadd = _r(2, 16, seed=3)
    got2 = FR.finalize(y, amax, 8, chan_add=cadd)
    ref2 = (FT.per_channel(y.permute(0, 3, 1, 2).contiguous(), 8).float() + cadd.float()[:, :, None, None]).half()
    assert torch.equal(got2, ref2.permute(0, 2, 3, 1))


def test_geglu_deinterleave_and_linear_amax():
    x = _r(64, 32, seed=4)
    w = _r(64, 32, seed=5, scale=0.2)   # [hidden 32 | gate 32]
    b = _r(64, seed=6, scale=0.1)
    half = 32
    idx = torch.arange(half).view(-1, 16)
    perm = torch.stack([idx, idx + half], 1).reshape(-1)
    outs = FR.linear(dict(x2d=x, weight=w[perm], wfmt="f16", bias=b[perm], geglu=True), None)
    y = F.linear(x.float(), w.float(), b.float()).half()
    h, g = y.chunk(2, dim=-1)
    ref = (h.float() * F.gelu(g.float()).half().float()).half()
    assert torch.equal(outs[0].ref, ref)
    res = _r(64, 64, seed=7)
    outs = FR.linear(dict(x2d=x, weight=w, wfmt="f16", bias=b, residual=res, amax=torch.zeros(2 * 64),
                          rows_per_sample=32, amax_post=True), None)
    fin = (y.float() + res.float()).half()
    assert torch.equal(outs[0].ref, fin)
    assert torch.equal(outs[1].ref, fin.float().abs().view(2, 32, 64).amax(1).reshape(-1))


def test_dequant_weight_codes():
    q = torch.randint(-8, 8, (4, 64), dtype=torch.int8)
    s = _r(4, 2, seed=8).abs()
    # qd_pack_int4 layout: per dword of 8 codes, nibble j = q(2j) + 8, nibble j + 4 = q(2j + 1) + 8
    c = (q.to(torch.int64) + 8).view(4, -1, 8)
    w = torch.zeros(c.shape[:2], dtype=torch.int64)
    for j in range(4):
        w |= c[..., 2 * j] << (4 * j)
        w |= c[..., 2 * j + 1] << (4 * j + 16)
    packed = torch.stack([(w >> (8 * i)) & 0xFF for i in range(4)], -1).reshape(4, -1).to(torch.uint8)
    w4 = FR.dequant_weight(packed, "i4", s, 32, None)
    w8 = FR.dequant_weight(q, "i8", s, 32, None)
    ref = (q.float() * s.float().repeat_interleave(32, 1)).half()
    assert torch.equal(w4, ref) and torch.equal(w8, ref)


def test_compare_bounds():
    r = _r(100, seed=9)
    assert FR.compare(r.clone(), FR.Out("y", r, ulps=0))[2] == 0
    bumped = r.clone()
    bumped[3] = (bumped[3].float() + FR.ulp(bumped[3:4]).float()[0] * 3).half()
    assert FR.compare(bumped, FR.Out("y", r, ulps=0))[2] == 1
    assert FR.compare(bumped, FR.Out("y", r, ulps=2))[2] == 1
    assert FR.compare(bumped, FR.Out("y", r, ulps=4))[2] == 0


def test_groupnorm_chain_quantized():
    x = _r(2, 8, 8, 64, seed=10, scale=2)
    gm, bt = (1 + 0.1 * _r(64, seed=11).float()).half(), (0.1 * _r(64, seed=12).float()).half()
    outs = FR.groupnorm_nhwc(dict(x=x, x2=None, fq_in=None, groups=32, eps=1e-5, gamma=gm, beta=bt, silu=True,
                                  q_bits=8), None)
    g16 = F.group_norm(x.float().permute(0, 3, 1, 2), 32, gm.float(), bt.float(), 1e-5).half()
    ref = FT.per_channel(F.silu(g16.float()).half(), 8).permute(0, 2, 3, 1)
    assert torch.equal(outs[0].ref, ref)
