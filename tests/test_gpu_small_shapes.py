"""The small-shape kernels of round 6: the weight-stream GEMV's SiLU epilogue (the
time-embedding activations at M <= 4), the narrow-output 3x3 conv (conv_out, Co <= 16) and the
one-launch per-channel fake-quant of a small NHWC tensor (conv_in's latent).

Tolerances: the GEMV / conv against fp32 torch on the same fp16 operands within 2 fp16 ulp + the
fp32 summation-order bound 4 sqrt(K) 2^-24 sum |x||w| (oracle/fused_ref.py's rule); the SiLU epilogue
bit-identical to silu() on the GEMV output; the fake-quant bit-exact to the golden-pinned numpy
oracle (fake_quant.py:123-131)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fake_quant_np as FQ

pytestmark = pytest.mark.gpu


def K():
    from qdiff import kernels
    return kernels


def ulp16(x):
    a = x.abs().clamp(min=6.1e-5)
    return torch.pow(2.0, torch.floor(torch.log2(a)) - 10)


def check_sum(got, ref32, absum, k, what):
    """|got - half(ref32)| <= 2 ulp + 4 sqrt(k) 2^-24 sum|x||w| elementwise."""
    got, ref32, absum = got.float().cpu(), ref32.float().cpu(), absum.float().cpu()
    ref = ref32.half().float()
    bound = 2 * ulp16(ref) + 4.0 * math.sqrt(k) * 2.0 ** -24 * absum
    err = (got - ref).abs()
    assert torch.isfinite(got).all(), what
    bad = int((err > bound).sum())
    assert bad == 0, f"{what}: {bad} / {err.numel()} outside; max err / bound {(err / bound).max().item():.3g}"


def _w_operand(k, w16, fmt, group):
    """(codes or fp16 weight, fmt, scales, group, fp16 dequantized buffer) via qd_weight_quant."""
    if fmt == "f16":
        return w16, "f16", None, 0, w16
    bits = 8 if fmt == "i8" else 4
    codes, sc, wdq = k.weight_quant(w16, group, bits)
    if fmt == "i4":
        codes = k.pack_int4(codes)
    return codes, fmt, sc, group, wdq


@pytest.mark.parametrize("M", [2, 4])
@pytest.mark.parametrize("fmt", ["f16", "i8", "i4"])
@pytest.mark.parametrize("N,Kd", [(1280, 320), (1280, 1280), (2048, 2816)])
def test_gemv_silu_epilogue(M, fmt, N, Kd, dev):
    k = K()
    g = torch.Generator().manual_seed(M * 7 + N + Kd)
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(N, Kd, generator=g) / math.sqrt(Kd)).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    r = torch.randn(M, N, generator=g).half().to(dev)
    assert k.gemv_shape(M, Kd, 0)
    wop, f, sc, gr, wdq = _w_operand(k, w, fmt, 64)
    y = k.linear(x, wop, f, sc, gr, bias=b)
    ref = x.float() @ wdq.float().t() + b.float()
    absum = x.float().abs() @ wdq.float().abs().t()
    check_sum(y, ref, absum, Kd, f"gemv M {M} {fmt}")
    # SiLU epilogue (residual first): bit-identical to linear -> silu on the same GEMV
    y2 = k.linear(x, wop, f, sc, gr, bias=b, residual=r)
    ys = k.linear(x, wop, f, sc, gr, bias=b, residual=r, silu=True)
    assert torch.equal(ys.view(torch.int16), k.silu(y2).view(torch.int16))


def test_silu_epilogue_needs_gemv_shape(dev):
    k = K()
    assert not k.gemv_shape(8, 320, 0)  # M 5..8 stay on the tile GEMM (an 8-row GEMV was slower)
    x = torch.randn(8, 320, device=dev).half()
    w = torch.randn(320, 320, device=dev).half()
    with pytest.raises(ValueError):
        k.linear(x, w, silu=True)


def test_temb_chain_gemv_silu(dev):
    """run_linear(..., silu=True) equals the two-launch form at M 4 (GEMV epilogue) and M 8 (tile GEMM
    + SiLU pass)."""
    from qdiff.unet import run_linear
    g = torch.Generator().manual_seed(3)
    lin = torch.nn.Linear(320, 1280).half().to(dev)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(1280, 320, generator=g) / 18).half())
    for m in (4, 8):
        x = torch.randn(m, 320, generator=g).half().to(dev)
        a = run_linear(lin, x, silu=True)
        b = K().silu(run_linear(lin, x))
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("n,h,w,ci,co,amax", [
    (8, 64, 64, 320, 8, True),      # SD1.5 conv_out (4 real channels + 4 zero-weight pad)
    (2, 33, 128, 128, 16, True),    # odd H, two 64-pixel segments per row
    (1, 16, 64, 64, 8, False),      # bias only (real channels 0-3, zero-weight pad 4-7)
])
def test_conv_narrow(n, h, w, ci, co, amax, dev):
    k = K()
    g = torch.Generator().manual_seed(n * 100 + h + co)
    x = torch.randn(n, h, w, ci, generator=g).half().to(dev)
    wt = (torch.randn(co, ci, 3, 3, generator=g) / math.sqrt(9 * ci)).half()
    if co == 8:
        wt[4:] = 0  # the UNet's co_pad rows
    b = (torch.randn(co, generator=g) * 0.1).half()
    if co == 8:
        b[4:] = 0
    wk = k.conv_weight_khwc(wt.to(dev).contiguous(), ci)
    am = torch.zeros(n * co, dtype=torch.float32, device=dev) if amax else None
    y = k.conv2d_nhwc(x, wk, ci, 1, 1, bias=b.to(dev), amax=am)
    xc = x.float().permute(0, 3, 1, 2).cpu()
    ref = F.conv2d(xc, wt.float(), b.float(), 1, 1).permute(0, 2, 3, 1)
    absum = F.conv2d(xc.abs(), wt.float().abs(), None, 1, 1).permute(0, 2, 3, 1)
    check_sum(y, ref, absum, 9 * ci, f"narrow conv {n}x{h}x{w} {ci}->{co}")
    if amax:
        got_am = y.float().abs().reshape(n, -1, co).amax(dim=1).reshape(-1)
        assert torch.equal(am, got_am), "amax epilogue != max |output|"


@pytest.mark.parametrize("n,h,w,c,cv", [(8, 64, 64, 8, 4), (2, 32, 32, 16, 0), (3, 16, 16, 64, 0), (1, 8, 8, 8, 8)])
def test_act_fq_small_bit_exact(n, h, w, c, cv, dev):
    k = K()
    g = torch.Generator().manual_seed(n + h + c)
    x = (torch.randn(n, h, w, c, generator=g) * 3).half()
    if cv:
        x[..., cv:] = 0
    xd = x.to(dev)
    assert k.act_fq_small_ok(xd)
    y = k.act_fq_nhwc_small(xd, 8, c_valid=cv).cpu()
    ref = FQ.quantize_activation_per_channel_absmax(x.permute(0, 3, 1, 2).numpy(), 8)
    ref = torch.from_numpy(np.ascontiguousarray(ref)).permute(0, 2, 3, 1)
    if cv:
        ref[..., cv:] = x[..., cv:]
    assert torch.equal(y.view(torch.int16), ref.contiguous().view(torch.int16))
    # and the two-pass form on the same input
    two = k.act_apply_nhwc(xd, k.act_absmax(xd, "per_channel", k.NHWC), 8, c_valid=cv).cpu()
    assert torch.equal(y.view(torch.int16), two.view(torch.int16))


@pytest.mark.parametrize("fmt", ["f16", "i8", "i4"])
@pytest.mark.parametrize("N,Kd,silu", [(1280, 320, True), (1280, 1280, True), (20160, 1280, False)])
def test_gemv_row_replicating_epilogue(fmt, N, Kd, silu, dev):
    """QD_EPI_ROWREP: one input row, the GEMV's output row stored to every row of [R, N] - each row
    bit-identical to the one-row call."""
    k = K()
    g = torch.Generator().manual_seed(N + Kd)
    x = torch.randn(1, Kd, generator=g).half().to(dev)
    w = (torch.randn(N, Kd, generator=g) / math.sqrt(Kd)).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    wop, f, sc, gr, _ = _w_operand(k, w, fmt, 64)
    one = k.linear(x, wop, f, sc, gr, bias=b, silu=silu)
    rep = k.linear(x, wop, f, sc, gr, bias=b, silu=silu, rep_rows=8)
    assert rep.shape == (8, N)
    assert torch.equal(rep.view(torch.int16), one.expand(8, N).contiguous().view(torch.int16))


def test_gemv_row_replicating_rejects(dev):
    k = K()
    w = torch.randn(1280, 320, device=dev).half()
    with pytest.raises(ValueError):
        k.linear(torch.randn(2, 320, device=dev).half(), w, rep_rows=8)
    with pytest.raises(ValueError):
        k.linear(torch.randn(1, 320, device=dev).half(), w, residual=torch.zeros(1, 1280, device=dev).half(),
                 rep_rows=8)


@pytest.mark.parametrize("qc", [None, dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)])
def test_unet_shared_time_embedding(qc, dev):
    """UNet fwd(temb_shared=True) - the denoising loops' one-timestep batch: the time embedding on
    row 0 and the stacked time_emb_proj stored to every row - against the batched form: every
    resnet's projection row within the GEMMs' summation-order bound (GEMV vs tile GEMM, through two
    SiLUs), all rows identical; and the whole eval against the oracle under test_gpu_unet's
    self-calibrated criterion."""
    import test_gpu_unet as TU
    from oracle.unet_ref import RefUNet
    k = K()
    model = TU._model(seed=3)
    unet = model.pipeline.unet
    cfg = unet.config
    sd = {kk: v.detach().cpu() for kk, v in unet.state_dict().items()}
    if qc is not None:
        model.quantize(quant_config=dict(qc), quantUnet=True)
    B = 8
    ts = torch.tensor([601.0], device=dev)
    temb = k.timestep_embedding(ts, None, B, cfg.block_out_channels[0])
    shared = unet._shared_temb(temb)
    assert shared is not None
    t = unet.time_embedding
    from qdiff.unet import run_linear
    batched = unet.temb_projections(run_linear(t.linear_2, run_linear(t.linear_1, temb, silu=True), silu=True))
    assert shared.keys() == batched.keys()
    for rid, a in shared.items():
        a, bb = a.float().cpu(), batched[rid].float().cpu()
        assert (a == a[:1]).all(), "rows of the shared projection differ"
        err = (a - bb).abs()
        tol = 8 * ulp16(bb) + 1e-3 * bb.abs().max()
        assert (err <= tol).all(), (err / tol).max().item()
    # the whole eval (the loop's form) against the oracle
    g = torch.Generator().manual_seed(13)
    x = torch.randn(B, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    ctx = torch.randn(B, 77, cfg.cross_attention_dim, generator=g).half()
    kv = unet.prepare_context(ctx.to(dev))
    out = unet.fwd(k.nchw_to_nhwc(x.to(dev), 8), temb, kv, temb_shared=True)
    got = k.nhwc_to_nchw(out, 4).cpu()
    q = None if qc is None else dict(qc)
    ref = RefUNet(TU._cfgdict(cfg), sd, q).forward(x, 601, ctx)
    ref32 = RefUNet(TU._cfgdict(cfg), sd, q, variant="fp32").forward(x, 601, ctx)
    TU._check_parity(got, ref, ref32, f"tiny UNet shared-temb eval {qc}")
