"""HIP kernels vs the golden-pinned oracle (bit-exact for the fake-quant math) and vs fp32 torch
references for the floating-point kernels (GEMM / conv / attention / norms), with the
tolerance stated in each test.  Runs on the MI355X (-m gpu)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fake_quant_np as FQ
from oracle import fake_quant_torch as FT
from oracle.unet_ref import ddim_step, timestep_embedding

pytestmark = pytest.mark.gpu


def K():
    from qdiff import kernels
    return kernels


def same_bits(a, b):
    a = np.ascontiguousarray(a, dtype=np.float16)
    b = np.ascontiguousarray(b, dtype=np.float16)
    return a.shape == b.shape and np.array_equal(a.view(np.uint16), b.view(np.uint16))


def ulp16(x):
    """fp16 ulp of |x| (x float32 tensor)."""
    a = x.abs().clamp(min=6.1e-5)
    return torch.pow(2.0, torch.floor(torch.log2(a)) - 10)


def assert_fp16_close(got, ref, ulps=2.0, atol=1e-3, frac=1.0):
    """|got - ref| <= ulps * ulp16(ref) + atol for at least `frac` of the elements."""
    got = got.float().cpu()
    ref = ref.float().cpu()
    ok = (got - ref).abs() <= ulps * ulp16(ref) + atol
    assert torch.isfinite(got).all()
    assert ok.float().mean().item() >= frac, f"{(~ok).sum().item()} / {ok.numel()} outside tolerance; " \
        f"max err {(got - ref).abs().max().item():.4g}"


# ------------------------------------------------------------------ fake-quant: bit-exact
def test_act_quant_bit_exact(golden, dev):
    k = K()
    g = golden["fake_quant_golden"]
    for bits in (4, 8, 16):
        x = torch.from_numpy(g[f"atok_b{bits}_in"]).to(dev)
        assert same_bits(k.act_fakequant(x, "per_token", bits).cpu().numpy(), g[f"atok_b{bits}_out"])
        x = torch.from_numpy(g[f"achan_b{bits}_in"]).to(dev)
        assert same_bits(k.act_fakequant(x, "per_channel", bits, layout=k.NCHW).cpu().numpy(), g[f"achan_b{bits}_out"])
        # NHWC path on the transposed tensor
        xh = x.permute(0, 2, 3, 1).contiguous()
        yh = k.act_fakequant(xh, "per_channel", bits, layout=k.NHWC).permute(0, 3, 1, 2).cpu().numpy()
        assert same_bits(yh, g[f"achan_b{bits}_out"])
        x = torch.from_numpy(g[f"aten_b{bits}_in"]).to(dev)
        assert same_bits(k.act_fakequant(x, "per_tensor", bits).cpu().numpy(), g[f"aten_b{bits}_out"])
        x = torch.from_numpy(g[f"agrp_b{bits}_in"]).to(dev)
        assert same_bits(k.act_fakequant(x, "per_group", bits, layout=k.NCHW, group=6).cpu().numpy(),
                         g[f"agrp_b{bits}_out"])


def test_public_quant_functions(golden, dev):
    import qdiff
    g = golden["fake_quant_golden"]
    for bits in (4, 8):
        for kk in (320, 768, 5120):
            w = torch.from_numpy(g[f"wgroup_b{bits}_k{kk}_in"]).to(dev)
            assert same_bits(qdiff.quantize_weight_absmax(w, bits, 128).cpu().numpy(), g[f"wgroup_b{bits}_k{kk}_out"])
        w = torch.from_numpy(g[f"wpc_b{bits}_64x32x3x3_in"]).to(dev)
        assert same_bits(qdiff.quantize_weight_per_channel_absmax(w, bits).cpu().numpy(), g[f"wpc_b{bits}_64x32x3x3_out"])
        w = torch.from_numpy(g[f"wpt_b{bits}_in"]).to(dev)
        assert same_bits(qdiff.quantize_weight_per_tensor_absmax(w, bits).cpu().numpy(), g[f"wpt_b{bits}_out"])
    x = torch.from_numpy(g["agrp_b8_in"]).to(dev)
    assert same_bits(qdiff.quantize_activation_per_channel_group_absmax(x, 8, 8).cpu().numpy(), g["agrp_b8_out"])


def test_weight_codes(golden, dev):
    k = K()
    g = golden["fake_quant_golden"]
    for bits in (4, 8):
        w = g[f"wgroup_b{bits}_k2560_in"]
        codes, scales, wdq = k.weight_quant(torch.from_numpy(w).to(dev), 128, bits)
        c_ref, s_ref, _ = FQ.quantize_weight_absmax_codes(w, bits, 128)
        assert np.array_equal(codes.cpu().numpy(), c_ref)
        assert same_bits(scales.cpu().numpy(), s_ref)
        assert same_bits(wdq.cpu().numpy(), g[f"wgroup_b{bits}_k2560_out"])
        if bits == 4:
            # qd_pack_int4: per little-endian dword of 8 codes, nibble j = q(2j) + 8 and
            # nibble j + 4 = q(2j + 1) + 8 (offset binary, k pairs in MFMA fragment order)
            packed = k.pack_int4(codes).cpu().numpy()
            w = packed.reshape(packed.shape[0], -1, 4).astype(np.uint32)
            w = w[..., 0] | (w[..., 1] << 8) | (w[..., 2] << 16) | (w[..., 3] << 24)
            sh = np.array([0, 16, 4, 20, 8, 24, 12, 28], dtype=np.uint32)
            q = ((w[..., None] >> sh) & 0xF).astype(np.int8) - 8
            assert np.array_equal(q.reshape(c_ref.shape), c_ref)


def test_fq_finalize_bit_exact(dev):
    k = K()
    rng = np.random.default_rng(3)
    y = (rng.standard_normal((2, 8, 8, 64)) * 3).astype(np.float16)
    res = rng.standard_normal((2, 8, 8, 64)).astype(np.float16)
    yt = torch.from_numpy(y).to(dev)
    amax = k.act_absmax(yt, "per_channel", k.NHWC)
    out = k.fq_finalize(yt, amax, 8, residual=torch.from_numpy(res).to(dev)).cpu().numpy()
    ref = FQ.quantize_activation_per_channel_absmax(y.transpose(0, 3, 1, 2), 8).transpose(0, 2, 3, 1)
    ref = (ref.astype(np.float32) + res.astype(np.float32)).astype(np.float16)
    assert same_bits(out, ref)
    cadd = rng.standard_normal((2, 64)).astype(np.float16)
    out2 = k.fq_finalize(yt, amax, 8, chan_add=torch.from_numpy(cadd).to(dev)).cpu().numpy()
    ref2 = FQ.quantize_activation_per_channel_absmax(y.transpose(0, 3, 1, 2), 8).transpose(0, 2, 3, 1)
    ref2 = (ref2.astype(np.float32) + cadd[:, None, None, :].astype(np.float32)).astype(np.float16)
    assert same_bits(out2, ref2)


def test_smooth_fold_and_hook(golden, dev):
    k = K()
    s = golden["smooth_golden"]
    lnw = torch.from_numpy(s["ln_w_in"]).to(dev)
    lnb = torch.from_numpy(s["ln_b_in"]).to(dev)
    fcs = [torch.from_numpy(s[f"fc{i}_w_in"]).to(dev) for i in range(3)]
    k.smooth_fold(lnw, lnb, fcs, torch.from_numpy(s["act"]).to(dev), 0.8)
    # f64 pow on device, rounded like torch's Half pow: every bit equal to the reference
    assert same_bits(lnw.cpu().numpy(), s["ln_w_out"])
    assert same_bits(lnb.cpu().numpy(), s["ln_b_out"])
    for i in range(3):
        assert same_bits(fcs[i].cpu().numpy(), s[f"fc{i}_w_out"])
    x = torch.from_numpy(s["hook_x"].reshape(-1, 320)).to(dev)
    ws = torch.empty(320, dtype=torch.float32, device=dev)
    sm = torch.zeros(320, dtype=torch.float32, device=dev)
    am = torch.empty(320, dtype=torch.float16, device=dev)
    k.channel_absmax_accum(x, ws, sm, am)
    k.channel_absmax_accum(x, ws, sm, None)
    assert same_bits(am.cpu().numpy(), s["hook_amax"])
    assert torch.equal(sm.cpu(), 2 * torch.from_numpy(s["hook_amax"]).float())


# ------------------------------------------------------------------ GEMMs vs fp32 torch
@pytest.mark.parametrize("M,N,Kd", [(128, 128, 64), (200, 320, 320), (616, 640, 768), (4096, 2560, 320),
                                    (8, 1280, 1280), (1000, 64, 128), (256, 1280, 5120), (512, 320, 640)])
@pytest.mark.parametrize("fmt", ["f16", "i8", "i4"])
def test_linear_formats(M, N, Kd, fmt, dev):
    k = K()
    g = torch.Generator().manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, generator=g).half()
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half()
    b = torch.randn(N, generator=g).half()
    res = torch.randn(M, N, generator=g).half()
    bits = {"f16": 8, "i8": 8, "i4": 4}[fmt]
    gs = FQ.shrink_group(Kd, 128)
    codes, scales, wdq = k.weight_quant(w.to(dev), gs, bits)
    if fmt == "f16":
        op, sc, grp = wdq, None, 0
    elif fmt == "i8":
        op, sc, grp = codes, scales, gs
    else:
        op, sc, grp = k.pack_int4(codes), scales, gs
    y = k.linear(x.to(dev), op, fmt, sc, grp, bias=b.to(dev), residual=res.to(dev)).cpu().float()
    pre = (x.float() @ wdq.cpu().float().t() + b.float()).half().float()
    yf = (pre + res.float()).half().float()
    # fp32 accumulation order differs -> the fp16 rounding of y = x.W + b may move by 1 ulp of
    # |y| (then the residual add rounds once more): |err| <= 1 ulp(|y|) + 1 ulp(|out|) + 1e-3
    tol = ulp16(pre) + ulp16(yf) + 1e-3
    assert ((y - yf).abs() <= tol).all(), (y - yf).abs().max().item()


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,Kd", [(4864, 2432), (1280, 320), (64, 4096), (8, 64), (640, 8192), (1536, 192)])
@pytest.mark.parametrize("fmt", ["f16", "i8", "i4"])
def test_linear_skinny_m_gemv(M, N, Kd, fmt, dev):
    """M <= 4 runs the skinny-M GEMV (k_gemv: weight-stream bound, register-resident activations)
    where K / 32 chunks fit its register budget (M 3-4 at K 8192 falls back to the tile GEMM):
    same dequant and epilogue rounding as the tile kernels, fp32 sums in another order."""
    k = K()
    g = torch.Generator().manual_seed(7 * M + N + Kd)
    x = torch.randn(M, Kd, generator=g).half()
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half()
    b = torch.randn(N, generator=g).half()
    res = torch.randn(M, N, generator=g).half()
    bits = {"f16": 8, "i8": 8, "i4": 4}[fmt]
    gs = FQ.shrink_group(Kd, 128) if Kd % 32 == 0 else Kd
    codes, scales, wdq = k.weight_quant(w.to(dev), gs, bits)
    op, sc, grp = {"f16": (wdq, None, 0), "i8": (codes, scales, gs), "i4": (k.pack_int4(codes), scales, gs)}[fmt]
    y = k.linear(x.to(dev), op, fmt, sc, grp, bias=b.to(dev), residual=res.to(dev)).cpu().float()
    pre = (x.float() @ wdq.cpu().float().t() + b.float()).half().float()
    yf = (pre + res.float()).half().float()
    tol = ulp16(pre) + ulp16(yf) + 1e-3
    assert ((y - yf).abs() <= tol).all(), (y - yf).abs().max().item()
    yt = k.linear(x.to(dev), op, fmt, sc, grp, bias=b.to(dev), gelu_tanh=True).cpu().float()
    ref_t = torch.nn.functional.gelu(pre, approximate="tanh").half().float()
    # a 1-ulp move of pre moves gelu_tanh(pre) by at most ~1.13 ulp(pre), then one more rounding
    tol_t = 1.2 * ulp16(pre) + ulp16(ref_t) + 1e-3
    assert ((yt - ref_t).abs() <= tol_t).all(), (yt - ref_t).abs().max().item()


def test_geglu_epilogue_packed_gelu_bit_exact(dev):
    """The GEMM epilogue's packed-fp32 GELU (gelu2_f) equals the scalar gelu_f of the standalone
    GEGLU kernel bit for bit on every finite fp16 gate value: an exact identity projection
    ([h | g] = x) feeds both, h = 1."""
    k = K()
    allg = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16).view(torch.float16)
    allg = allg[torch.isfinite(allg)]
    n = (allg.numel() + 63) // 64 * 64
    g = torch.zeros(n, dtype=torch.float16)
    g[: allg.numel()] = allg
    M, I = n // 64, 64
    x = torch.cat([torch.ones(M, I, dtype=torch.float16), g.view(M, I)], 1).to(dev)  # K = 128
    w = torch.zeros(2 * I, 2 * I, dtype=torch.float16)
    w[torch.arange(2 * I), torch.arange(2 * I)] = 1.0
    w = w.to(dev)
    y = k.linear(x, w, "f16")
    assert torch.equal(y, x)
    perm = k.geglu_interleave_rows(2 * I, dev)
    fused = k.linear(x, w[perm].contiguous(), "f16", geglu=True)
    unfused = k.geglu(y)
    assert torch.equal(fused, unfused)


@pytest.mark.parametrize("M,I,Kd,fmt", [(256, 1280, 320, "f16"), (1000, 640, 640, "i8"), (64, 2560, 1280, "i4")])
def test_linear_geglu_epilogue(M, I, Kd, fmt, dev):
    k = K()
    g = torch.Generator().manual_seed(M + I)
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(2 * I, Kd, generator=g) / Kd ** 0.5).half().to(dev)
    b = torch.randn(2 * I, generator=g).half().to(dev)
    gs = FQ.shrink_group(Kd, 128)
    codes, scales, wdq = k.weight_quant(w, gs, 4 if fmt == "i4" else 8)
    if fmt == "f16":
        op, sc, grp = wdq, None, 0
    elif fmt == "i8":
        op, sc, grp = codes, scales, gs
    else:
        op, sc, grp = k.pack_int4(codes), scales, gs
    perm = k.geglu_interleave_rows(2 * I, dev)
    fused = k.linear(x, op[perm].contiguous(), fmt, None if sc is None else sc[perm].contiguous(), grp,
                     bias=b[perm].contiguous(), geglu=True).cpu().float()
    y = k.linear(x, op, fmt, sc, grp, bias=b)
    unfused = k.geglu(y).cpu().float()
    pre = (x.float().cpu() @ wdq.cpu().float().t() + b.float().cpu()).half().float()
    h, gt = pre.chunk(2, -1)
    ref = (h * F.gelu(gt).half().float()).half().float()
    # same accumulation -> identical up to the planner's tile choice (1-ulp of the projection)
    # a 1-ulp move of h or g propagates as ulp(h)*|gelu(g)| + |h|*ulp(g)*|gelu'(g)| (gelu' <= 1.13)
    tol = 2 * ulp16(ref) + 2 * ulp16(h) * gt.abs() + 2.5 * h.abs() * ulp16(gt) + 1e-3
    assert ((fused - ref).abs() <= tol).all(), (fused - ref).abs().max().item()
    assert ((fused - unfused).abs() <= tol).all()


def test_linear_amax_epilogue(dev):
    k = K()
    g = torch.Generator().manual_seed(1)
    M, N, Kd = 4 * 256, 320, 640
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(N, Kd, generator=g) / 25).half().to(dev)
    amax = torch.empty(4 * N, dtype=torch.float32, device=dev)
    y = k.linear(x, w, "f16", amax=amax, rows_per_sample=256)
    ref = y.float().abs().view(4, 256, N).amax(1).reshape(-1)
    assert torch.equal(amax, ref)


@pytest.mark.parametrize("cin,cout,ksz,stride,hw,ups", [(64, 64, 3, 1, 16, False), (64, 128, 3, 2, 16, False),
                                                        (128, 64, 1, 1, 8, False), (4, 64, 3, 1, 16, False),
                                                        (64, 64, 3, 1, 8, True), (320, 320, 3, 1, 32, False),
                                                        (960, 320, 3, 1, 16, False), (1280, 1280, 3, 1, 8, False),
                                                        (640, 640, 3, 1, 16, False)])
def test_conv_nhwc(cin, cout, ksz, stride, hw, ups, dev):
    k = K()
    g = torch.Generator().manual_seed(cin * 7 + cout)
    n = 2
    x = torch.randn(n, cin, hw, hw, generator=g).half()
    w = (torch.randn(cout, cin, ksz, ksz, generator=g) / (cin * ksz * ksz) ** 0.5).half()
    b = torch.randn(cout, generator=g).half()
    cip = (cin + 7) // 8 * 8
    xh = k.nchw_to_nhwc(x.to(dev), cip)
    wk = k.conv_weight_khwc(w.to(dev), cip)
    pad = ksz // 2
    amax = torch.empty(n * cout, dtype=torch.float32, device=dev)
    y = k.conv2d_nhwc(xh, wk, cin, stride, pad, ups, bias=b.to(dev), amax=amax)
    xin = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if ups else x.float()
    ref = F.conv2d(xin, w.float(), b.float(), stride, pad).half().float()
    got = k.nhwc_to_nchw(y).cpu().float()
    assert_fp16_close(got, ref, ulps=2.0, atol=1e-3)
    assert torch.equal(amax.view(n, cout).cpu(), got.abs().amax(dim=(2, 3)))
    # deterministic (split-K slabs are reduced in a fixed order)
    y2 = k.conv2d_nhwc(xh, wk, cin, stride, pad, ups, bias=b.to(dev), amax=amax)
    assert torch.equal(y, y2)


def test_gemm_plans_split_k_for_small_m():
    from qdiff import _lib
    lib = _lib.load()
    # SD1.5 8x8 level: M = 8 * 64, N = 1280, K = 9 * 1280 -> too few 128-row tiles, K is split
    assert lib.qd_gemm_workspace(512, 1280, 11520, 0, 0, 64, 4) > 0
    assert lib.qd_gemm_workspace(128, 1280, 11520, 0, 0, 64, 4) > 0
    # the big-M levels run unsplit
    assert lib.qd_gemm_workspace(32768, 320, 2880, 0, 0, 4096, 4) == 0


# ------------------------------------------------------------------ attention
@pytest.mark.parametrize("b,heads,sq,skv,d", [(2, 8, 256, 256, 40), (2, 8, 64, 77, 80), (1, 8, 128, 77, 160),
                                              (2, 5, 200, 200, 64), (1, 2, 4096, 4096, 40), (4, 8, 4000, 333, 40),
                                              (4, 8, 4096, 1024, 80), (2, 4, 1024, 1024, 64), (1, 3, 600, 333, 64)])
def test_attention(b, heads, sq, skv, d, dev):
    k = K()
    g = torch.Generator().manual_seed(sq + skv + d)
    c = heads * d
    q = torch.randn(b, sq, c, generator=g).half()
    kk = torch.randn(b, skv, c, generator=g).half()
    v = torch.randn(b, skv, c, generator=g).half()
    o = k.attention(q.to(dev), kk.to(dev), v.to(dev), heads).cpu().float()
    qh = q.float().view(b, sq, heads, d).transpose(1, 2)
    kh = kk.float().view(b, skv, heads, d).transpose(1, 2)
    vh = v.float().view(b, skv, heads, d).transpose(1, 2)
    p = torch.softmax(qh @ kh.transpose(-1, -2) / math.sqrt(d), -1)
    ref = (p @ vh).transpose(1, 2).reshape(b, sq, c)
    # P is rounded to fp16 before P.V (flash-style); error ~ 1e-3 relative to |V|
    assert (o - ref).abs().max().item() < 1e-2


@pytest.mark.parametrize("b,heads,sq,skv,d", [(2, 2, 256, 40, 40), (2, 2, 300, 77, 40), (1, 2, 256, 192, 40),
                                              (2, 3, 520, 333, 40), (1, 2, 512, 4096, 40), (2, 2, 256, 256, 80)])
def test_attention_stagger_bit_identical(b, heads, sq, skv, d, dev):
    """Round 6: the 8-wave 32x32x16 kernel with the half-tile stagger between SIMD partners
    (qd_attn_force 8; the heuristic's choice) runs the same operations per query in the same order
    as the unstaggered form (force 9): identical bits at 1 / 2 / odd / even key-tile counts."""
    from qdiff import _lib
    k = K()
    g = torch.Generator().manual_seed(sq * 7 + skv + d)
    c = heads * d
    q = torch.randn(b, sq, c, generator=g).half().to(dev)
    kk = (torch.randn(b, skv, c, generator=g) * 2).half().to(dev)
    v = torch.randn(b, skv, c, generator=g).half().to(dev)
    lib = _lib.load()
    try:
        lib.qd_attn_force(8)
        o8 = k.attention(q, kk, v, heads)
        lib.qd_attn_force(9)
        o9 = k.attention(q, kk, v, heads)
    finally:
        lib.qd_attn_force(0)
    assert torch.equal(o8.view(torch.int16), o9.view(torch.int16))


@pytest.mark.parametrize("d,gain", [(40, 3.0), (80, 2.5), (64, 3.0), (160, 2.5)])
def test_attention_sharp_softmax(d, gain, dev):
    """large-norm Q / K (logits of magnitude 30-60, a near one-hot softmax).  The kernel
    multiplies Q by scale * log2(e) and rounds it to fp16 before the QK^T MFMA, so each logit carries
    an extra relative error <= 2^-11 of sum_i |q_i k_i| * scale; a softmax with logit errors <= e moves
    its output by <= 2 e max|v| (to first order).  The bound below is that term + the 1e-2 of the
    fp16 P rounding (test_attention), against an fp32 reference of the same fp16 inputs."""
    k = K()
    g = torch.Generator().manual_seed(d)
    b, heads, sq, skv = 2, 4, 512, 640
    c = heads * d
    q = (torch.randn(b, sq, c, generator=g) * gain).half()
    kk = (torch.randn(b, skv, c, generator=g) * gain).half()
    v = torch.randn(b, skv, c, generator=g).half()
    o = k.attention(q.to(dev), kk.to(dev), v.to(dev), heads).cpu().float()
    qh = q.float().view(b, sq, heads, d).transpose(1, 2)
    kh = kk.float().view(b, skv, heads, d).transpose(1, 2)
    vh = v.float().view(b, skv, heads, d).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(d)
    assert s.abs().max().item() > 25  # sharp
    ref = (torch.softmax(s, -1) @ vh).transpose(1, 2).reshape(b, sq, c)
    e_logit = 2.0 ** -11 * (qh.abs() @ kh.abs().transpose(-1, -2)).amax(-1) / math.sqrt(d)  # [b, h, sq]
    bound = 1e-2 + 2 * e_logit * vh.abs().amax(dim=(-1, -2), keepdim=True)[..., 0]
    err = (o - ref).abs().view(b, sq, heads, d).amax(-1).transpose(1, 2)  # [b, h, sq]
    print(f"d={d}: max err {err.max().item():.3g}, max bound {bound.max().item():.3g}, "
          f"max err/bound {(err / bound).max().item():.3f}")
    assert (err <= bound).all()


# ------------------------------------------------------------------ norms / elementwise
@pytest.mark.parametrize("c,hw,silu,q", [(320, 64, True, 8), (640, 256, True, 0), (960, 16, True, 8),
                                         (64, 256, False, 8), (2560, 16, True, 4)])
def test_groupnorm_fused(c, hw, silu, q, dev):
    k = K()
    g = torch.Generator().manual_seed(c + hw)
    n = 2
    x = (torch.randn(n, c, hw, generator=g) * 2 + 0.5).half()
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half()
    bet = (0.1 * torch.randn(c, generator=g)).half()
    xh = x.transpose(1, 2).contiguous().to(dev)  # NHWC [n, hw, c]
    y = k.groupnorm_nhwc(xh, 32, 1e-5, gam.to(dev), bet.to(dev), silu=silu, q_bits=q)
    ref = F.group_norm(x.view(n, c, hw, 1), 32, gam, bet, 1e-5)
    if silu:
        ref = F.silu(ref)
    got = y.cpu().transpose(1, 2).reshape(n, c, hw, 1)
    if q:
        ref = FT.per_channel(ref, q)
        # a 1-ulp GN difference can flip one rounding step of the fake-quant grid
        step = ref.float().abs().amax(dim=(2, 3), keepdim=True) / (2 ** (q - 1) - 1)
        err = (got.float() - ref.float()).abs()
        assert (err <= step * 1.01 + 1e-3).all()
        assert (err <= 1e-3).float().mean() > 0.995
    else:
        assert_fp16_close(got, ref, ulps=2.0, atol=2e-3)


@pytest.mark.parametrize("c,hw,silu,q", [(320, 4096, True, 8), (640, 1024, True, 8), (960, 1024, False, 8),
                                         (1280, 1024, True, 8), (640, 4096, True, 0),
                                         (128, 1024, True, 8)])  # 4 channels per group: per-channel shifts
def test_groupnorm_streaming_path(c, hw, silu, q, dev):
    """hw > 256: the two streaming passes (statistics -> coefficients -> apply) against torch,
    with channels whose tiny gamma / negative beta keep the SiLU output below the extremes
    bound (the fallback amax scan)."""
    k = K()
    g = torch.Generator().manual_seed(c + hw + q)
    n = 2
    x = (torch.randn(n, c, hw, generator=g) * 2 + 0.5).half()
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half()
    bet = (0.1 * torch.randn(c, generator=g)).half()
    gam[::37] = 0.01
    bet[::37] = -0.5
    xh = x.transpose(1, 2).contiguous().to(dev)
    ref = F.group_norm(x.view(n, c, hw, 1), 32, gam, bet, 1e-5)
    if silu:
        ref = F.silu(ref)
    if q:
        ref = FT.per_channel(ref, q)
    y = k.groupnorm_nhwc(xh, 32, 1e-5, gam.to(dev), bet.to(dev), silu=silu, q_bits=q)
    assert torch.equal(y, k.groupnorm_nhwc(xh, 32, 1e-5, gam.to(dev), bet.to(dev), silu=silu, q_bits=q))
    got = y.cpu().transpose(1, 2).reshape(n, c, hw, 1)
    if q:
        step = ref.float().abs().amax(dim=(2, 3), keepdim=True) / (2 ** (q - 1) - 1)
        err = (got.float() - ref.float()).abs()
        assert (err <= step * 1.01 + 1e-3).all()
        assert (err <= 1e-3).float().mean() > 0.995
    else:
        assert_fp16_close(got, ref, ulps=2.0, atol=2e-3)


@pytest.mark.parametrize("rps,c,bits", [(4096, 320, 8), (1024, 640, 8), (256, 1280, 8), (64, 1280, 4)])
def test_layernorm_fq_equals_finalize_then_layernorm(rps, c, bits, dev):
    """The fused proj_in output fake-quant + norm1 (qd_layernorm_fq) writes the same residual
    stream and LayerNorm output as qd_fq_finalize followed by qd_layernorm, bit for bit."""
    k = K()
    g = torch.Generator().manual_seed(rps + c)
    n = 2
    y = (torch.randn(n, rps, c, generator=g) * 3).half().to(dev)
    amax = y.float().abs().amax(1).reshape(-1).contiguous()
    amax[::7] *= 0.5  # some channels clip
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half().to(dev)
    bet = (0.1 * torch.randn(c, generator=g)).half().to(dev)
    t_ref = k.fq_finalize(y, amax, bits)
    h_ref = k.layernorm(t_ref.view(-1, c), 1e-5, gam, bet)
    t, h = k.layernorm_fq(y.view(-1, c), amax, bits, rps, 1e-5, gam, bet)
    assert torch.equal(t, t_ref.view(-1, c))
    assert torch.equal(h, h_ref)


@pytest.mark.parametrize("hw,c,q,silu,temb", [(1024, 640, 8, True, False), (4096, 320, 8, True, False),
                                              (1024, 320, 0, False, False), (4096, 320, 8, False, False),
                                              (4096, 320, 8, True, True), (1024, 640, 8, True, True)])
def test_groupnorm_fin_equals_finalize_then_groupnorm(hw, c, q, silu, temb, dev):
    """GroupNorm on a pending block output (conv output + output fake-quant + residual add): the
    materialised x and the GroupNorm output equal fq_finalize followed by groupnorm_nhwc, bit for
    bit (tiny-gamma channels exercise the fallback amax scan, which reads the raw sources)."""
    k = K()
    g = torch.Generator().manual_seed(hw + c + q)
    n = 2
    y = (torch.randn(n, hw, c, generator=g) * 1.5).half().to(dev)
    r = torch.randn(n, hw, c, generator=g).half().to(dev)
    amax = y.float().abs().amax(dim=1).reshape(-1).contiguous()
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half()
    bet = (0.1 * torch.randn(c, generator=g)).half()
    gam[::37] = 0.01
    bet[::37] = -0.5
    gam, bet = gam.to(dev), bet.to(dev)
    if temb:  # conv1 -> norm2: + the time-embedding projection per (n, c) (a row-strided view)
        big = (torch.randn(n, 3 * c, generator=g) * 0.3).half().to(dev)
        cadd = big[:, c: 2 * c]
        x_ref = k.fq_finalize(y, amax, 8, chan_add=cadd)
        h_ref = k.groupnorm_nhwc(x_ref, 32, 1e-5, gam, bet, silu=silu, q_bits=q)
        x, h = k.groupnorm_fin(y, amax, 8, None, 32, 1e-5, gam, bet, silu=silu, q_bits=q, cadd=cadd)
        # and the fq_in path (both passes recompute the transform) gives the same output
        assert torch.equal(k.groupnorm_nhwc(y, 32, 1e-5, gam, bet, silu=silu, q_bits=q, fq_in=(amax, 8, cadd)), h_ref)
    else:
        x_ref = k.fq_finalize(y, amax, 8, residual=r)
        h_ref = k.groupnorm_nhwc(x_ref, 32, 1e-5, gam, bet, silu=silu, q_bits=q)
        x, h = k.groupnorm_fin(y, amax, 8, r, 32, 1e-5, gam, bet, silu=silu, q_bits=q)
    assert torch.equal(x, x_ref)
    assert torch.equal(h, h_ref)


def test_groupnorm_two_sources(dev):
    k = K()
    g = torch.Generator().manual_seed(5)
    a = torch.randn(2, 64, 640, generator=g).half()
    b2 = torch.randn(2, 64, 320, generator=g).half()
    gam = torch.ones(960).half()
    bet = torch.zeros(960).half()
    y1 = k.groupnorm_nhwc(a.to(dev), 32, 1e-5, gam.to(dev), bet.to(dev), silu=True, x2=b2.to(dev))
    y2 = k.groupnorm_nhwc(k.concat_c(a.to(dev), b2.to(dev)), 32, 1e-5, gam.to(dev), bet.to(dev), silu=True)
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("hw,c1,c2", [(4096, 640, 320), (1024, 1280, 640), (300, 320, 320), (4096, 320, 320)])
def test_groupnorm_xamax_feeds_concat_quant(hw, c1, c2, dev):
    """qd_groupnorm_xamax: the up blocks' norm1 over the skip concat also returns the input's exact
    per-(n, c) max |x| (channel extremes of its statistics pass); the shortcut's input quant from it
    (qd_act_apply_cat_nhwc) equals qd_act_quant_cat_nhwc (its own column-max pass) bit for bit, and
    the GroupNorm output is unchanged."""
    k = K()
    g = torch.Generator().manual_seed(hw + c1)
    n = 2
    a = (torch.randn(n, hw, c1, generator=g) * 2).half().to(dev)
    b2 = (torch.randn(n, hw, c2, generator=g) * 3).half().to(dev)
    b2[1, :, 7] = 0  # an all-zero channel (amax clamp)
    c = c1 + c2
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half().to(dev)
    bet = (0.1 * torch.randn(c, generator=g)).half().to(dev)
    y0 = k.groupnorm_nhwc(a, 32, 1e-5, gam, bet, silu=True, q_bits=8, x2=b2)
    y1, xam = k.groupnorm_nhwc(a, 32, 1e-5, gam, bet, silu=True, q_bits=8, x2=b2, want_xamax=True)
    assert torch.equal(y0, y1)
    exact = torch.cat([a, b2], -1).float().abs().amax(1).reshape(-1)
    assert torch.equal(xam, exact)
    assert torch.equal(k.act_apply_cat_nhwc(a, b2, 8, xam), k.act_quant_cat_nhwc(a, b2, 8))


@pytest.mark.parametrize("rows,c", [(77, 320), (4096, 640), (33, 1280), (5, 2048), (8195, 320), (20001, 160), (3, 3072)])
def test_layernorm(rows, c, dev):
    k = K()
    g = torch.Generator().manual_seed(rows + c)
    x = (torch.randn(rows, c, generator=g) * 3).half()
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half()
    bet = (0.1 * torch.randn(c, generator=g)).half()
    y = k.layernorm(x.to(dev), 1e-5, gam.to(dev), bet.to(dev)).cpu()
    ref = F.layer_norm(x.float(), (c,), gam.float(), bet.float(), 1e-5)
    assert_fp16_close(y, ref, ulps=2.0, atol=2e-3)


def test_elementwise(dev):
    k = K()
    g = torch.Generator().manual_seed(9)
    h = (torch.randn(300, 2 * 640, generator=g) * 2).half()
    out = k.geglu(h.to(dev)).cpu()
    a, gate = h.chunk(2, -1)
    ref = (a.float() * F.gelu(gate.float()).half().float()).half()
    assert_fp16_close(out, ref, ulps=1.0, atol=1e-3)
    x = (torch.randn(1000, generator=g) * 4).half()
    assert_fp16_close(k.silu(x.to(dev)).cpu(), F.silu(x.float()), ulps=1.0, atol=1e-4)
    y = torch.randn(1000, generator=g).half()
    assert torch.equal(k.add(x.to(dev), y.to(dev)).cpu(), (x.float() + y.float()).half())
    a2 = torch.randn(6, 5, 24, generator=g).half()
    b2 = torch.randn(6, 5, 40, generator=g).half()
    assert torch.equal(k.concat_c(a2.to(dev), b2.to(dev)).cpu(), torch.cat([a2, b2], -1))
    xn = torch.randn(2, 5, 7, 9, generator=g).half()
    xh = k.nchw_to_nhwc(xn.to(dev), 8)
    assert torch.equal(xh[..., :5].cpu(), xn.permute(0, 2, 3, 1)) and xh[..., 5:].abs().sum().item() == 0
    assert torch.equal(k.nhwc_to_nchw(xh, 5).cpu(), xn)


def test_timestep_embedding_and_ddim(dev):
    k = K()
    from qdiff.scheduler import ddim_tables
    ts, a_t, a_p = ddim_tables(50)
    ts_d = ts.float().to(dev)
    idx = torch.tensor([7], dtype=torch.int32, device=dev)
    e = k.timestep_embedding(ts_d, idx, 3, 320).cpu()
    ref = timestep_embedding(torch.full((3,), int(ts[7])), 320).half()
    assert_fp16_close(e, ref, ulps=1.0, atol=2e-3)
    # CFG + DDIM step
    g = torch.Generator().manual_seed(2)
    B, h, w = 2, 8, 8
    lat = torch.randn(B, 4, h, w, generator=g).half()
    eps = torch.randn(2 * B, 4, h, w, generator=g).half()
    lat_h = k.nchw_to_nhwc(lat.to(dev), 8)
    eps_h = k.nchw_to_nhwc(eps.to(dev), 8)
    nxt = torch.zeros(2 * B, h, w, 8, dtype=torch.float16, device=dev)
    step = torch.tensor([5], dtype=torch.int32, device=dev)
    k.cfg_ddim_step(lat_h, eps_h, 7.5, a_t.to(dev), a_p.to(dev), step, nxt, c=4)
    got = k.nhwc_to_nchw(lat_h, 4).cpu()
    ref = ddim_step(eps, 5, lat, a_t, a_p, 7.5)
    assert_fp16_close(got, ref, ulps=2.0, atol=1e-3)
    assert step.item() == 6
    assert torch.equal(k.nhwc_to_nchw(nxt[:B], 4), k.nhwc_to_nchw(nxt[B:], 4))


# ------------------------------------------------------------------ GEMM kernel families
@pytest.fixture
def forced_gemm():
    """Run every GEMM of the test on one qd_gemm_force id (kernels.force_gemm overrides the
    tuner's per-shape choice; -1 / None = tuned).  A variant that does not apply to a shape
    falls back to the library planner inside libqdiff."""
    from qdiff import kernels

    def force(v):
        kernels.force_gemm(None if v is None or v < 0 else v)
    yield force
    kernels.force_gemm(None)


@pytest.mark.parametrize("variant", [-1, 0, 1, 3] + list(range(100, 118)) + [300, 301]
                         # explicit split counts: the split-K reduction takes the post-residual amax
                         + [2104, 4105, 5110, 2117])
@pytest.mark.parametrize("fmt", ["f16", "i8"])
def test_linear_post_residual_amax(variant, fmt, forced_gemm, dev):
    """QD_EPI_AMAX_POST: the epilogue adds the residual to the fragments and reduces the
    per-(sample, column) amax of the FINAL output (the consuming conv's input amax).  Output as
    the plain residual epilogue's, amax equal to the exact max of that output (ping-pong plans
    fall back to unsplit tiles that support it; an explicit split count reduces it in
    k_splitk_reduce after the residual add)."""
    k = K()
    g = torch.Generator().manual_seed(11)
    M, N, Kd, rps = 4 * 1024, 320, 1280, 1024
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(dev)
    b = torch.randn(N, generator=g).half().to(dev)
    r = (torch.randn(M, N, generator=g) * 2).half().to(dev)
    if fmt == "i8":
        codes, scales, wdq = k.weight_quant(w, 128, 8)
        op, sc, grp, wf = codes, scales, 128, wdq
    else:
        op, sc, grp, wf = w, None, 0, None
    forced_gemm(variant)
    plain = k.linear(x, op, fmt, sc, grp, bias=b, residual=r, weight_f16=wf)
    amax = torch.full((M // rps * N,), 123.0, device=dev)  # the call zeroes it (amax_zeroed=False)
    got = k.linear(x, op, fmt, sc, grp, bias=b, residual=r, weight_f16=wf, amax=amax, rows_per_sample=rps,
                   amax_post=True)
    # (the two calls may take different split counts - another fp32 summation order: the outputs
    # agree to the fp16 rounding of the projection, an ulp of which can exceed an ulp of the
    # output where the residual cancels it)
    gc, pc, rc = got.cpu().float(), plain.cpu().float(), r.cpu().float()
    assert ((gc - pc).abs() <= 2 * ulp16(pc.abs() + rc.abs()) + 1e-3).all()
    ref = got.float().abs().view(M // rps, rps, N).amax(1).reshape(-1)
    assert torch.equal(amax, ref)


@pytest.mark.parametrize("variant", [0, 1, 2, 3] + list(range(100, 116)) + [200, 201, 202, 203, 300, 301, 302, 303, 304]
                         # + 1000 * s: an explicit split-K count s (1 = unsplit) for the DMA / ping-pong / halo plans
                         + [1100, 2104, 3109, 4105, 6114, 8115, 1301, 2301, 4301, 1202, 2202, 3203, 5203]
                         # explicit splits of tiles whose wave rows exceed a sample (the reduction makes the amax)
                         + [2103, 3113, 2117])
def test_gemm_variants_conv_and_linear(variant, forced_gemm, dev):
    """Every kernel family / tile (register-staged and LDS-DMA) on ragged shapes: rows past M,
    conv halo, stride 2, fused 2x upsample, the 4-channel conv_in (any-Ci decode), K tails,
    split-K, residual, amax and GEGLU epilogues."""
    k = K()
    forced_gemm(variant)
    g = torch.Generator().manual_seed(variant + 5)
    for cin, cout, ksz, stride, hw, ups, n in ((64, 320, 3, 1, 16, False, 2), (128, 128, 3, 2, 16, False, 1),
                                               (4, 64, 3, 1, 8, False, 2), (64, 64, 3, 1, 8, True, 1),
                                               (320, 640, 1, 1, 8, False, 3), (1280, 320, 3, 1, 8, False, 2)):
        x = torch.randn(n, cin, hw, hw, generator=g).half()
        w = (torch.randn(cout, cin, ksz, ksz, generator=g) / (cin * ksz * ksz) ** 0.5).half()
        b = torch.randn(cout, generator=g).half()
        cip = (cin + 7) // 8 * 8
        xh = k.nchw_to_nhwc(x.to(dev), cip)
        wk = k.conv_weight_khwc(w.to(dev), cip)
        amax = torch.empty(n * cout, dtype=torch.float32, device=dev)
        y = k.conv2d_nhwc(xh, wk, cin, stride, ksz // 2, ups, bias=b.to(dev), amax=amax)
        xin = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if ups else x.float()
        ref = F.conv2d(xin, w.float(), b.float(), stride, ksz // 2).half().float()
        got = k.nhwc_to_nchw(y).cpu().float()
        assert_fp16_close(got, ref, ulps=2.0, atol=1e-3)
        assert torch.equal(amax.view(n, cout).cpu(), got.abs().amax(dim=(2, 3))), (variant, cin, cout)
    for M, N, Kd in ((200, 320, 320), (616, 640, 776), (4096, 1280, 5120), (77, 256, 1280)):
        x = torch.randn(M, Kd, generator=g).half()
        w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half()
        b = torch.randn(N, generator=g).half()
        res = torch.randn(M, N, generator=g).half()
        y = k.linear(x.to(dev), w.to(dev), "f16", bias=b.to(dev), residual=res.to(dev)).cpu().float()
        pre = (x.float() @ w.float().t() + b.float()).half().float()
        yf = (pre + res.float()).half().float()
        assert ((y - yf).abs() <= ulp16(pre) + ulp16(yf) + 1e-3).all(), (variant, M, N, Kd)
    M, I, Kd = 300, 640, 320
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(2 * I, Kd, generator=g) / Kd ** 0.5).half().to(dev)
    b = torch.randn(2 * I, generator=g).half().to(dev)
    perm = k.geglu_interleave_rows(2 * I, dev)
    fused = k.linear(x, w[perm].contiguous(), "f16", bias=b[perm].contiguous(), geglu=True).cpu().float()
    pre = (x.float().cpu() @ w.cpu().float().t() + b.float().cpu()).half().float()
    h, gt = pre.chunk(2, -1)
    ref = (h * F.gelu(gt).half().float()).half().float()
    tol = 2 * ulp16(ref) + 2 * ulp16(h) * gt.abs() + 2.5 * h.abs() * ulp16(gt) + 1e-3
    assert ((fused - ref).abs() <= tol).all(), (variant, (fused - ref).abs().max().item())


@pytest.mark.parametrize("variant", [100, 101, 102, 103, 104, 105, 109, 110, 111, 112, 113, 114, 115, 116, 117,
                                     300, 301, 302, 303, 304])
def test_int4_lds_dma_variants_bit_identical(variant, forced_gemm, dev):
    """Packed-int4 codes through the LDS-DMA / ping-pong families (BDma4: codes + the K step's
    group-scale row DMA'd into the stage, dequantized per fragment) give the SAME bits as the
    same tile variant on the fp16 dequantized buffer: half(q * s) from LDS equals the buffer, and
    the K order (and split-K plan) is the variant's.  Ragged M / N tails, groups 32 / 64 / 128,
    split-K shapes, bias / residual / amax / GEGLU epilogues."""
    k = K()
    forced_gemm(variant)
    g = torch.Generator().manual_seed(variant)
    for M, N, Kd, gs in ((200, 320, 320, 64), (616, 640, 768, 128), (4096, 1280, 5120, 128), (77, 200, 1280, 128),
                         (1000, 2560, 320, 32), (4096, 320, 1280, 128), (128, 128, 64, 64), (300, 64, 128, 64)):
        x = torch.randn(M, Kd, generator=g).half().to(dev)
        w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(dev)
        b = torch.randn(N, generator=g).half().to(dev)
        res = torch.randn(M, N, generator=g).half().to(dev)
        codes, scales, wdq = k.weight_quant(w, gs, 4)
        packed = k.pack_int4(codes)
        y4 = k.linear(x, packed, "i4", scales, gs, bias=b, residual=res)
        y16 = k.linear(x, wdq, "f16", bias=b, residual=res)
        assert torch.equal(y4, y16), (variant, M, N, Kd, (y4.float() - y16.float()).abs().max().item())
        if M % 256 == 0:
            a4 = torch.empty(M // 256 * N, dtype=torch.float32, device=dev)
            a16 = torch.empty_like(a4)
            z4 = k.linear(x, packed, "i4", scales, gs, bias=b, amax=a4, rows_per_sample=256)
            z16 = k.linear(x, wdq, "f16", bias=b, amax=a16, rows_per_sample=256)
            assert torch.equal(z4, z16) and torch.equal(a4, a16), (variant, M, N, Kd)
    M, I, Kd, gs = 1000, 640, 320, 64
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(2 * I, Kd, generator=g) / Kd ** 0.5).half().to(dev)
    b = torch.randn(2 * I, generator=g).half().to(dev)
    perm = k.geglu_interleave_rows(2 * I, dev)
    codes, scales, wdq = k.weight_quant(w[perm].contiguous(), gs, 4)
    f4 = k.linear(x, k.pack_int4(codes), "i4", scales, gs, bias=b[perm].contiguous(), geglu=True)
    f16 = k.linear(x, wdq, "f16", bias=b[perm].contiguous(), geglu=True)
    assert torch.equal(f4, f16), variant


@pytest.mark.parametrize("bits,with_cadd,hw", [(8, True, 256), (0, True, 256), (8, False, 256), (4, True, 256),
                                               (8, True, 1024), (0, False, 1024)])
def test_groupnorm_fq_in_matches_finalize_then_norm(bits, with_cadd, hw, dev):
    """GroupNorm on a raw conv output with the output quant + temb add applied on the fly equals
    fq_finalize followed by GroupNorm, bit for bit; includes channels whose SiLU output stays
    below the extremes bound (tiny gamma, negative beta) so the fallback amax scan runs."""
    k = K()
    g = torch.Generator().manual_seed(bits * 3 + with_cadd + hw)
    n, c = 2, 640
    y = (torch.randn(n, hw, c, generator=g) * 1.5).half().to(dev)
    amax = y.float().abs().amax(dim=1).reshape(-1).contiguous() if bits else None
    big = (torch.randn(n, 3 * c, generator=g) * 0.3).half().to(dev)
    cadd = big[:, 100 * 8: 100 * 8 + c] if with_cadd else None  # row-strided view, like the stacked temb
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half()
    bet = (0.1 * torch.randn(c, generator=g)).half()
    gam[::37] = 0.01
    bet[::37] = -0.5
    gam, bet = gam.to(dev), bet.to(dev)
    fin = k.fq_finalize(y, amax, bits, chan_add=cadd)
    ref = k.groupnorm_nhwc(fin, 32, 1e-5, gam, bet, silu=True, q_bits=8)
    got = k.groupnorm_nhwc(y, 32, 1e-5, gam, bet, silu=True, q_bits=8, fq_in=(amax, bits, cadd))
    assert torch.equal(got, ref)
    # the fallback-scanned channels are quantized with their exact amax
    # (torch-CPU Half ops, the reference's op-boundary rounding, as test_groupnorm_fused)
    gn = F.group_norm(fin.cpu().transpose(1, 2).reshape(n, c, hw, 1), 32, gam.cpu(), bet.cpu(), 1e-5)
    ref2 = FT.per_channel(F.silu(gn), 8)
    got2 = got.cpu().transpose(1, 2).reshape(n, c, hw, 1)
    step = ref2.float().abs().amax(dim=(2, 3), keepdim=True) / 127
    err = (got2.float() - ref2.float()).abs()
    assert (err <= step * 1.01 + 1e-3).all(), err.max().item()
    assert (err <= 1e-3).float().mean() > 0.995


def test_act_quant_cat_matches_concat_then_quant(dev):
    k = K()
    g = torch.Generator().manual_seed(9)
    a = (torch.randn(2, 16, 16, 640, generator=g) * 3).half().to(dev)
    b2 = torch.randn(2, 16, 16, 320, generator=g).half().to(dev)
    got = k.act_quant_cat_nhwc(a, b2, 8)
    cat = k.concat_c(a, b2)
    ref = k.act_fakequant(cat, "per_channel", 8, layout=k.NHWC)
    assert torch.equal(got, ref)


def test_fast_reciprocal_fake_quant_is_exact(dev):
    """rcp_exact + fq_apply_r (all apply kernels) == the IEEE-division fake-quant, for every fp16
    scale and the values next to every quantization midpoint; and the f16 quotient of the shortcut
    == half(IEEE x / s) for every finite fp16 x (a 3-op f32 Markstein division from RN(1/s) was
    tried instead of the f64 product and failed this on 95229 of the ~4e9 pairs)."""
    from qdiff import _lib
    counts = torch.zeros(3, dtype=torch.int32, device=dev)
    _lib.call("qd_selftest_recip", counts.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert counts.tolist() == [0, 0, 0]


@pytest.mark.parametrize("variant", [200, 201, 202, 203, 204, 205])
def test_conv_halo_kernel(variant, forced_gemm, dev):
    """Halo-staged 3x3 conv: 16/32/64-wide images, fused 2x upsample, split-K over channel
    chunks (ragged 64-channel chunk counts), bias + amax + residual epilogues."""
    k = K()
    forced_gemm(variant)
    g = torch.Generator().manual_seed(variant)
    for cin, cout, hw, ups, n, res in ((128, 320, 16, False, 2, True), (320, 640, 32, False, 2, False),
                                       (192, 160, 64, False, 1, True), (64, 128, 16, True, 2, False),
                                       (1280, 1280, 16, False, 2, False)):
        x = torch.randn(n, cin, hw, hw, generator=g).half()
        w = (torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5).half()
        b = torch.randn(cout, generator=g).half()
        xh = k.nchw_to_nhwc(x.to(dev), cin)
        wk = k.conv_weight_khwc(w.to(dev), cin)
        H = 2 * hw if ups else hw
        r = torch.randn(n, H, H, cout, generator=g).half().to(dev) if res else None
        amax = torch.empty(n * cout, dtype=torch.float32, device=dev)
        y = k.conv2d_nhwc(xh, wk, cin, 1, 1, ups, bias=b.to(dev), residual=r, amax=amax)
        xin = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if ups else x.float()
        pre = F.conv2d(xin, w.float(), b.float(), 1, 1).half().float()
        got = k.nhwc_to_nchw(y).cpu().float()
        if res:
            ref = (pre + k.nhwc_to_nchw(r).cpu().float()).half().float()
            tol = ulp16(pre) + ulp16(ref) + 1e-3
            assert ((got - ref).abs() <= tol).all(), (variant, cin, cout, hw)
        else:
            assert_fp16_close(got, pre, ulps=2.0, atol=1e-3)
        # amax is of the pre-residual output (the conv output the reference fake-quantizes)
        assert torch.allclose(amax.view(n, cout).cpu(), pre.abs().amax(dim=(2, 3)), rtol=2e-3, atol=1e-3)


def test_conv_halo_split_phase_bit_identical(forced_gemm, dev):
    """The split-phase halo conv (202 / 203) changes only when tiles are loaded and read, not the K
    order: its outputs equal the lock-step halo kernel's (200 / 201) bit for bit, on the SD1.5 64x64 shape at
    full width (every pipeline position of a 5-chunk, 45-step K loop) and a split-K shape; so do its
    128-pixel tiles (204 / 205, images up to 32 wide: the same K order per output pixel)."""
    k = K()
    g = torch.Generator().manual_seed(31)
    for n, hw, cin, cout in ((8, 64, 320, 320), (2, 16, 1280, 1280), (2, 32, 640, 640), (8, 32, 640, 640)):
        x = torch.randn(n, hw, hw, cin, generator=g).half().to(dev)
        wk = (torch.randn(cout, 3, 3, cin, generator=g) / (cin * 9) ** 0.5).half().to(dev)
        b = torch.randn(cout, generator=g).half().to(dev)
        # (the 128-pixel tiles against the others at one explicit split count, 1000 * s + variant: the
        # planner's own split choice depends on the tile count)
        pairs = ((200, 202), (201, 203)) + (((1200, 1202, 1204), (1201, 1203, 1205)) if hw <= 32 else ())
        for vs in pairs:
            outs = []
            for v in vs:
                forced_gemm(v)
                amax = torch.empty(n * cout, dtype=torch.float32, device=dev)
                y = k.conv2d_nhwc(x, wk, cin, 1, 1, False, bias=b, amax=amax)
                outs.append((y, amax))
            for o, v in zip(outs[1:], vs[1:]):
                assert torch.equal(outs[0][0], o[0]), (n, hw, cin, cout, v)
                assert torch.equal(outs[0][1], o[1]), (n, hw, cin, cout, v)


@pytest.mark.parametrize("variant", [-1, 0, 100, 106, 300, 301, 303])
def test_linear_gelu_tanh_epilogue(variant, forced_gemm, dev):
    """SD3 FeedForward net.0: half(gelu_tanh(half(x W^T + b))) fused into the GEMM epilogue (also
    through the split-K reduce: K = 4096 at small M)."""
    k = K()
    forced_gemm(variant)
    g = torch.Generator().manual_seed(17)
    for M, N, Kd in ((300, 640, 320), (64, 512, 4096), (1024, 1280, 640)):
        x = torch.randn(M, Kd, generator=g).half()
        w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half()
        b = torch.randn(N, generator=g).half()
        y = k.linear(x.to(dev), w.to(dev), "f16", bias=b.to(dev), gelu_tanh=True).cpu().float()
        pre = (x.float() @ w.float().t() + b.float()).half()
        ref = F.gelu(pre.float(), approximate="tanh").half().float()
        # a 1-ulp move of the pre-activation propagates through gelu' <= 1.13
        tol = 1.13 * ulp16(pre.float()) + ulp16(ref) + 1e-3
        assert ((y - ref).abs() <= tol).all(), (variant, M, N, Kd, (y - ref).abs().max())


def test_cfg_pndm_step_bit_exact_vs_torch_pndm(dev):
    """CFG + PNDMScheduler.step_plms (skip_prk_steps) on device == the torch-CPU restatement in
    diffusers' op order (oracle/unet_ref.py PNDMRef), bit for bit, over every branch: the first
    step, the counter-1 restart, the 2-, 3- and 4-term multisteps and the final alpha."""
    from oracle.unet_ref import PNDMRef
    from qdiff.scheduler import pndm_tables
    k = K()
    steps = 8
    ts, a_t, a_p = pndm_tables(steps)
    g = torch.Generator().manual_seed(4)
    b, h, w, c, cp = 2, 8, 8, 4, 8
    lat0 = torch.randn(b, c, h, w, generator=g).half()
    lat = k.nchw_to_nhwc(lat0.to(dev), cp)
    ets = torch.zeros(4, *lat.shape, dtype=torch.float16, device=dev)
    cur = torch.zeros_like(lat)
    idx = torch.zeros(1, dtype=torch.int32, device=dev)
    at_d, ap_d = a_t.to(dev), a_p.to(dev)
    ref = PNDMRef(num_inference_steps=steps)
    rl = lat0
    for i in range(len(ts)):
        uo = (torch.randn(2 * b, c, h, w, generator=g) * 0.5).half()
        k.cfg_pndm_step(lat, k.nchw_to_nhwc(uo.to(dev), cp), 7.5, at_d, ap_d, idx, ets, cur, c=c)
        u, cc = uo.chunk(2)
        rl = ref.step(u + 7.5 * (cc - u), int(ts[i]), rl)
        got = k.nhwc_to_nchw(lat, c).cpu()
        assert same_bits(got.numpy(), rl.numpy()), (i, (got.float() - rl.float()).abs().max().item())


@pytest.mark.parametrize("M,Kd", [(4096, 320), (300, 320), (77, 1280), (32768, 320)])
@pytest.mark.parametrize("variant", [None, 118, 101, 112])
@pytest.mark.parametrize("bias,i8_out", [(True, False), (False, False), (True, True)])
def test_linear_ln_equals_linear_then_layernorm(M, Kd, variant, bias, i8_out, dev):
    """The row-complete LayerNorm epilogue (attn.to_out + residual -> norm2 / norm3 in one launch):
    y and h bit-identical to linear() followed by layernorm() / layernorm_i8(), every row-complete
    tile, ragged M (rows past M) included."""
    k = K()
    N = 320
    g = torch.Generator().manual_seed(M + Kd)
    x = torch.randn(M, Kd, generator=g).half().to(dev)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(dev)
    b = torch.randn(N, generator=g).half().to(dev) if bias else None
    r = (torch.randn(M, N, generator=g) * 3).half().to(dev)
    gamma = (1 + 0.1 * torch.randn(N, generator=g)).half().to(dev)
    beta = (0.1 * torch.randn(N, generator=g)).half().to(dev)
    assert k.linear_ln_ok(N) and not k.linear_ln_ok(640)
    k.force_gemm(variant)
    try:
        y, h = k.linear_ln(x, w, r, gamma, beta, 1e-5, bias=b, i8_out=i8_out)
    finally:
        k.force_gemm(None)
    # the reference linear unsplit (forced: 1100 = LDS-DMA tile, split count 1): every unsplit fp16
    # tile sums K in the same order, a tuned split-K choice for the shape would not
    k.force_gemm(1100)
    try:
        y0 = k.linear(x, w, "f16", bias=b, residual=r)
    finally:
        k.force_gemm(None)
    assert torch.equal(y, y0)
    if i8_out:
        q0, s0 = k.layernorm_i8(y0, 1e-5, gamma, beta)
        assert torch.equal(h[0], q0) and torch.equal(h[1], s0)
    else:
        assert torch.equal(h, k.layernorm(y0, 1e-5, gamma, beta))


@pytest.mark.parametrize("n,hw,ci,co,add", [(8, 8, 1280, 1280, "res"), (8, 16, 1280, 1280, "res"), (8, 8, 2560, 1280, "cadd"),
                                            (2, 16, 640, 640, "none"), (8, 32, 640, 640, "res"), (3, 8, 320, 640, "res")])
@pytest.mark.parametrize("variant", [None, 4100, 6104, 2202, 1100])
def test_conv2d_fq_equals_conv_then_finalize(n, hw, ci, co, add, variant, dev):
    """The quantized conv + output fake-quant + residual / time-embedding add as one call
    (qd_conv2d_fq: the split-K reduction finalizes the output where the plan splits): output and
    amax bit-identical to conv2d_nhwc(amax) + fq_finalize under every forced tile / split."""
    k = K()
    g = torch.Generator().manual_seed(n * hw + ci + co)
    x = torch.randn(n, hw, hw, ci, generator=g).half().to(dev)
    w = (torch.randn(co, 3, 3, ci, generator=g) / (9 * ci) ** 0.5).half().to(dev)
    b = torch.randn(co, generator=g).half().to(dev)
    res = torch.randn(n, hw, hw, co, generator=g).half().to(dev) if add == "res" else None
    cadd = torch.randn(n, co, generator=g).half().to(dev) if add == "cadd" else None
    k.force_gemm(variant)
    try:
        a0 = torch.zeros(n * co, dtype=torch.float32, device=dev)
        y0 = k.conv2d_nhwc(x, w, ci, 1, 1, bias=b, amax=a0)
        x0 = k.fq_finalize(y0, a0, 8, residual=res, chan_add=cadd)
        a1 = torch.zeros(n * co, dtype=torch.float32, device=dev)
        xam = torch.full((n * co,), -1.0, dtype=torch.float32, device=dev)
        x1 = k.conv2d_fq(x, w, ci, 8, a1, 1, 1, bias=b, residual=res, chan_add=cadd, xamax=xam)
    finally:
        k.force_gemm(None)
    assert torch.equal(a0, a1)
    assert torch.equal(x0.view(torch.int16), x1.view(torch.int16))
    # the consumer conv's per-channel input amax, reduced by the same launch: exactly act_absmax
    assert torch.equal(xam, k.act_absmax(x0, "per_channel", k.NHWC))
