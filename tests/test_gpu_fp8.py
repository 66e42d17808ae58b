"""W4A8-fp8 mode for SD3.5 (quantize(..., fp8_act=True); BASELINE config C5's "fp8 activations on
CDNA4"): the HIP kernels against oracle/fp8_ref.py.

Per-token e4m3 codes and scales, and the W4 codes' e4m3 form, are bit-exact targets (torch's
float8_e4m3fn conversion is the oracle).  The GEMM (v_mfma_scale_f32_16x16x128_f8f6f4 per
128-code group, group scale applied to each MFMA result) is compared with the float64 group sum
within 1 fp16 ulp + the fp32 accumulation bound, and every tile variant gives identical bits (no
split-K; the K order is fixed).  Model level: a tiny MMDiT in the fp8 mode against the oracle
MMDiT in the same mode (self-calibrated rule of tests/test_gpu_mmdit.py), and the mode's stated
accuracy against W4A16 at SD3.5-Large width."""
import dataclasses

import pytest
import torch

from oracle import fp8_ref as F8R

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_quant_rows_fp8_bit_exact():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(1)
    for m, k in ((333, 2432), (64, 9728), (7, 128), (1, 4096)):
        x = (torch.randn(m, k, generator=g) * torch.exp(torch.randn(m, 1, generator=g))).half()
        x[0, :] = 0
        if m > 2:
            x[2, 5] = 60000.0
        q, s = K.quant_rows_fp8(x.to(DEV))
        rq, rs = F8R.quant_rows_fp8(x)
        assert torch.equal(s.cpu(), rs), (m, k)
        assert torch.equal(q.cpu(), rq), (m, k, int((q.cpu() != rq).sum()))


def test_fp8_weight_conversion_exact():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(2)
    codes = torch.randint(-8, 8, (320, 2432), generator=g).to(torch.int8)
    scales = (torch.rand(320, 19, generator=g) * 0.01 + 1e-4).half()
    w8, gs = K.fp8_weight(codes.to(DEV), scales.to(DEV), 128)
    assert torch.equal(F8R.decode(w8.cpu()), codes.float())
    assert torch.equal(gs.cpu(), scales.float().t().contiguous())


def _gemm_case(seed, m, n, k, bias=True):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(m, k, generator=g) * 2).half()
    codes = torch.randint(-8, 8, (n, k), generator=g).to(torch.int8)
    scales = (torch.rand(n, k // 128, generator=g) * 0.02 + 1e-3).half()
    b = (torch.randn(n, generator=g) * 0.1).half() if bias else None
    return x, codes, scales, b


@pytest.mark.parametrize("m,n,k", [(8192, 2432, 2432), (666, 7296, 2432), (8192, 9728, 2432), (8192, 2432, 9728),
                                   (100, 264, 256)])
def test_linear_fp8_matches_oracle_all_variants(m, n, k):
    from qdiff import kernels as K
    x, codes, scales, b = _gemm_case(m + n + k, m, n, k)
    xq, sa = F8R.quant_rows_fp8(x)
    v, yref, mag = F8R.linear_fp8(xq, sa, codes, scales, 128, b)
    w8, gs = K.fp8_weight(codes.to(DEV), scales.to(DEV), 128)
    xqd, sad = xq.to(DEV), sa.to(DEV)
    outs = []
    try:
        for var in K.F8_VARIANTS:
            K.force_gemm(var)
            outs.append(K.linear_fp8(xqd, sad, w8, gs, bias=b.to(DEV)).cpu())
    finally:
        K.force_gemm(None)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    got = outs[0].double()
    # 1 fp16 ulp of the result + the accumulation error, measured against the |terms| sum: the
    # scaled fp8 MFMA's internal sum of 128 products is not an IEEE fp32 chain (measured
    # max err / sum|terms| printed below; bound 2^-16 of it)
    err = (got - v).abs()
    rel_mag = float(((err - v.abs() * 2.0 ** -11).clamp(min=0) / mag.clamp(min=1e-30)).max())
    print(f"fp8 GEMM M{m} N{n} K{k}: max excess error / sum|terms| = {rel_mag:.3g} (2^{torch.tensor(max(rel_mag, 1e-30)).log2().item():.1f})")
    bound = v.abs() * 2.0 ** -10 + mag * 2.0 ** -16 + 1e-6
    bad = err > bound
    assert not bad.any(), (int(bad.sum()), float(err.max()))
    assert (got == yref.double()).double().mean() > 0.9


def test_linear_fp8_epilogues():
    from qdiff import kernels as K
    x, codes, scales, b = _gemm_case(9, 4096, 512, 1024)
    xq, sa = F8R.quant_rows_fp8(x)
    v, _, mag = F8R.linear_fp8(xq, sa, codes, scales, 128, b)
    w8, gs = K.fp8_weight(codes.to(DEV), scales.to(DEV), 128)
    res = torch.randn(4096, 512).half()
    y = K.linear_fp8(xq.to(DEV), sa.to(DEV), w8, gs, bias=b.to(DEV), residual=res.to(DEV)).cpu()
    base = K.linear_fp8(xq.to(DEV), sa.to(DEV), w8, gs, bias=b.to(DEV)).cpu()
    assert torch.equal(y, (base.float() + res.float()).half())
    gt = K.linear_fp8(xq.to(DEV), sa.to(DEV), w8, gs, bias=b.to(DEV), gelu_tanh=True).cpu()
    ref = torch.nn.functional.gelu(base.float(), approximate="tanh").half()
    ulp = torch.clamp(ref.float().abs(), min=2.0 ** -14) * 2.0 ** -10
    d = (gt.float() - ref.float()).abs()
    assert (d <= 2 * ulp + 2e-7).all(), float(d.max())
    assert (d == 0).float().mean() > 0.95


def _cfgdict(cfg):
    return {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}


def _rel(got, ref):
    got, ref = got.float().cpu(), ref.float().cpu()
    s = ref.abs().max().item()
    d = (got - ref).abs()
    return d.max().item() / s, d.mean().item() / s


def _one_eval(model, x, t, enc, pooled):
    from qdiff import kernels as K
    tr = model.pipeline.transformer
    prep = tr.prepare_context(enc.to(DEV), pooled.to(DEV))
    temb = K.timestep_embedding(torch.tensor([float(t)], device=DEV), None, x.shape[0], 256)
    return K.nhwc_to_nchw(tr.fwd(K.nchw_to_nhwc(x.to(DEV), x.shape[1]), temb, prep), x.shape[1]).cpu()


def test_tiny_mmdit_fp8_eval_matches_oracle():
    from oracle.mmdit_ref import RefMMDiT
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    from qdiff.models import StableDiffusion3_5
    from qdiff.pipeline_io import QDiffPipeline
    cfg = tiny_mmdit_config(num_layers=3, num_attention_heads=2, attention_head_dim=64, joint_attention_dim=128,
                            caption_projection_dim=128, pooled_projection_dim=128)
    tr = SD3Transformer2DModel(cfg).half().init_synthetic(4).to(DEV)
    sd = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    model = StableDiffusion3_5(QDiffPipeline(transformer=tr, class_name="StableDiffusion3Pipeline"),
                               "StableDiffusion3Pipeline", False, {}, None)
    qc = dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False)
    model.quantize(quant_config=dict(qc), quantTransformer=True, fp8_act=True)
    n_f8 = sum(1 for m in tr.modules() if getattr(m, "fp8_act", False))
    assert n_f8 > 0
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, cfg.in_channels, cfg.sample_size, cfg.sample_size, generator=g).half()
    enc = torch.randn(2, 77, cfg.joint_attention_dim, generator=g).half()
    pooled = torch.randn(2, cfg.pooled_projection_dim, generator=g).half()
    got = _one_eval(model, x, 777.0, enc, pooled)
    ref = RefMMDiT(_cfgdict(cfg), sd, dict(qc), fp8=True).forward(x, 777.0, enc, pooled)
    ref32 = RefMMDiT(_cfgdict(cfg), sd, dict(qc), variant="fp32", fp8=True).forward(x, 777.0, enc, pooled)
    assert len(RefMMDiT(_cfgdict(cfg), sd, dict(qc), fp8=True).f8) >= n_f8
    smx, smean = _rel(ref32, ref)
    mx, mean = _rel(got, ref)
    mx32, mean32 = _rel(got, ref32)
    print(f"tiny MMDiT W4A8-fp8 ({n_f8} fp8 linears): gpu-vs-half {mx:.4g}/{mean:.4g} gpu-vs-fp32 {mx32:.4g}/"
          f"{mean32:.4g} spread {smx:.4g}/{smean:.4g}")
    tmx, tmean = 1.5 * smx + 2e-3, 1.5 * smean + 2e-3
    assert mx <= tmx and mean <= tmean and mx32 <= tmx and mean32 <= tmean


@pytest.mark.timeout(600)
def test_sd35_large_width_fp8_accuracy_vs_w4a16():
    """Stated accuracy of the mode at SD3.5-Large width (2 blocks, 512^2, 333-token context):
    the W4A8-fp8 eval against the same model's W4A16 eval (both on the GPU)."""
    import dataclasses as dc
    from qdiff.mmdit import SD35_LARGE, SD3Transformer2DModel
    from qdiff.models import StableDiffusion3_5
    from qdiff.pipeline_io import QDiffPipeline
    cfg = dc.replace(SD35_LARGE, num_layers=2, sample_size=64)
    outs = {}
    g = torch.Generator().manual_seed(13)
    x = torch.randn(2, cfg.in_channels, 64, 64, generator=g).half()
    enc = torch.randn(2, 333, cfg.joint_attention_dim, generator=g).half()
    pooled = torch.randn(2, cfg.pooled_projection_dim, generator=g).half()
    for fp8 in (False, True):
        with torch.device(DEV):
            tr = SD3Transformer2DModel(cfg).half()
        tr.init_synthetic(7, rng_device=DEV)
        model = StableDiffusion3_5(QDiffPipeline(transformer=tr, class_name="StableDiffusion3Pipeline"),
                                   "StableDiffusion3Pipeline", False, {}, None)
        model.quantize(quant_config=dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
                       quantTransformer=True, fp8_act=fp8)
        outs[fp8] = _one_eval(model, x, 974.1, enc, pooled)
        del model, tr
        torch.cuda.empty_cache()
    mx, mean = _rel(outs[True], outs[False])
    print(f"SD3.5-L width, 2 blocks: W4A8-fp8 vs W4A16 max {mx:.4g} mean {mean:.4g}")
    assert torch.isfinite(outs[True].float()).all()
    assert mx <= 0.15 and mean <= 0.02, (mx, mean)


def test_fp8_mode_save_load_roundtrip(tmp_path):
    """save_quantized / from_quantized keep the fp8 mode (rebuilt from the stored W4 codes)."""
    from qdiff.models import StableDiffusion3_5
    model = StableDiffusion3_5.from_pretrained("synthetic:sd35-tiny", device=DEV, seed=5)
    model.quantize(quant_config=dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
                   quantTransformer=True, fp8_act=True)
    cfg = model.pipeline.transformer.config
    model.save_quantized(str(tmp_path))
    re = StableDiffusion3_5.from_quantized(str(tmp_path), "StableDiffusion3Pipeline")
    assert re.fp8_act
    n1 = sum(1 for m in model.pipeline.transformer.modules() if getattr(m, "fp8_act", False))
    n2 = sum(1 for m in re.pipeline.transformer.modules() if getattr(m, "fp8_act", False))
    assert n1 == n2 > 0
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, cfg.in_channels, cfg.sample_size, cfg.sample_size, generator=g).half()
    enc = torch.randn(2, 40, cfg.joint_attention_dim, generator=g).half()
    pooled = torch.randn(2, cfg.pooled_projection_dim, generator=g).half()
    assert torch.equal(_one_eval(model, x, 401.0, enc, pooled), _one_eval(re, x, 401.0, enc, pooled))
