"""SD3 / SD3.5 MMDiT on the GPU vs the CPU oracle (oracle/mmdit_ref.py).

Op-level: the elementwise MMDiT kernels match torch-CPU Half ops bit-exactly where the op is a
single fp16 rounding of an exactly computed value (gated residual, position add, copies,
unpatchify, CFG + flow-match step), and within 1-2 fp16 ulp where an fp32 reduction or a
transcendental is involved (adaLN LayerNorm, RMSNorm, GELU-tanh).  Model-level: the same
self-calibrated criterion as tests/test_gpu_unet.py (GPU vs oracle within 1.5 x the oracle's own
fp16-vs-fp32 spread + 2e-3, max and mean relative to max|ref|).  Parity of the diffusers
architecture itself is unpinned.
"""
import dataclasses

import pytest
import torch
import torch.nn.functional as F

from oracle.mmdit_ref import RefMMDiT, denoise, euler_step, flowmatch_tables

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _cfgdict(cfg):
    return {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}


def _rel_errs(got, ref):
    got, ref = got.float().cpu(), ref.float().cpu()
    scale = ref.abs().max().item()
    d = (got - ref).abs()
    return d.max().item() / scale, d.mean().item() / scale


def _check_parity(got, ref, ref32, what):
    smx, smean = _rel_errs(ref32, ref)
    mx, mean = _rel_errs(got, ref)
    mx32, mean32 = _rel_errs(got, ref32)
    print(f"{what}: gpu-vs-half max {mx:.4g} mean {mean:.4g} | gpu-vs-fp32 max {mx32:.4g} mean {mean32:.4g} | "
          f"oracle spread max {smx:.4g} mean {smean:.4g}")
    tmx, tmean = 1.5 * smx + 2e-3, 1.5 * smean + 2e-3
    assert mx <= tmx and mean <= tmean, (mx, mean, tmx, tmean)
    assert mx32 <= tmx and mean32 <= tmean, (mx32, mean32, tmx, tmean)


def _ulp_close(got, ref, ulps=2):
    got, ref = got.float().cpu(), ref.float().cpu()
    ulp = torch.clamp(ref.abs(), min=2.0 ** -14) * 2.0 ** -10
    bad = (got - ref).abs() > ulps * ulp + 1e-6
    assert not bad.any(), f"{int(bad.sum())} elements beyond {ulps} ulp; max diff {(got - ref).abs().max().item()}"


def _model(name="synthetic:sd35-tiny", seed=0):
    from qdiff.models import StableDiffusion3_5
    return StableDiffusion3_5.from_pretrained(name, device=DEV, seed=seed)


def _inputs(cfg, seed, b=1, sc=40):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(2 * b, cfg.in_channels, cfg.sample_size, cfg.sample_size, generator=g).half()
    enc = torch.randn(2 * b, sc, cfg.joint_attention_dim, generator=g).half()
    pooled = torch.randn(2 * b, cfg.pooled_projection_dim, generator=g).half()
    return x, enc, pooled


def _one_eval(model, x, t, enc, pooled):
    from qdiff import kernels as K
    tr = model.pipeline.transformer
    prep = tr.prepare_context(enc.to(DEV), pooled.to(DEV))
    xh = K.nchw_to_nhwc(x.to(DEV), x.shape[1])
    ts = torch.tensor([float(t)], device=DEV)
    temb = K.timestep_embedding(ts, None, x.shape[0], 256)
    out = tr.fwd(xh, temb, prep)
    return K.nhwc_to_nchw(out, x.shape[1]).cpu()


# ------------------------------------------------------------------ op level
def test_adaln_and_gated_residual():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(1)
    for b, s, c in ((2, 64, 128), (2, 40, 2432), (1, 333, 1536), (3, 7, 8)):
        x = (torch.randn(b * s, c, generator=g) * 3).half()
        mod = (torch.randn(b, 6 * c, generator=g) * 0.5).half()
        shift, scale, gate = mod[:, :c], mod[:, c:2 * c], mod[:, 2 * c:3 * c]
        ref = (F.layer_norm(x.float(), (c,), eps=1e-6).half().view(b, s, c) * (1 + scale[:, None])
               + shift[:, None]).view(b * s, c)
        md = mod.to(DEV)
        got = K.adaln(x.to(DEV), s, shift=md[:, :c], scale=md[:, c:2 * c])
        # a 1-ulp LayerNorm difference (fp32 reduction order) propagates through the modulation:
        # bound it by the ulp of the product term, not of the (possibly cancelled) result
        prod = (F.layer_norm(x.float(), (c,), eps=1e-6).view(b, s, c) * (1 + scale.float()[:, None])).view(b * s, c)
        err = (got.float().cpu() - ref.float()).abs()
        assert (err <= 2.0 ** -10 * (prod.abs() + ref.float().abs()) * 1.01 + 1e-6).all(), (b, s, c, err.max())
        assert (err == 0).float().mean() > 0.99
        y = (torch.randn(b * s, c, generator=g)).half()
        refg = (x.view(b, s, c) + gate.unsqueeze(1) * y.view(b, s, c)).view(b * s, c)
        gotg = K.gated_residual(x.to(DEV), y.to(DEV), md[:, 2 * c:3 * c], s)
        assert torch.equal(gotg.cpu(), refg), (b, s, c)


def test_rmsnorm_heads_grouped_rows_and_gelu_tanh():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(2)
    n, s, sc, heads = 2, 64, 40, 3
    for d in (64, 128, 32):
        c = heads * d
        L = s + sc
        J = (torch.randn(n, L, 3 * c, generator=g) * 2).half()
        w = (torch.rand(d, generator=g) + 0.5).half()
        Jd = J.to(DEV)
        K.rmsnorm_heads(Jd[:, :, c:], n * s, heads, d, 3 * c, w.to(DEV), 1e-6, rows_per_group=s, group_stride=L)
        ref = J.clone()
        kx = ref[:, :s, c:2 * c].reshape(n, s, heads, d)
        var = kx.float().pow(2).mean(-1, keepdim=True)
        ref[:, :s, c:2 * c] = ((kx * torch.rsqrt(var + 1e-6)).half() * w).reshape(n, s, c)
        got = Jd.cpu()
        _ulp_close(got, ref)
        assert torch.equal(got[:, s:], J[:, s:]) and torch.equal(got[:, :, :c], J[:, :, :c])
    x = (torch.randn(4096, generator=g) * 4).half()
    _ulp_close(K.gelu_tanh(x.to(DEV)), F.gelu(x.float(), approximate="tanh").half(), ulps=1)


def test_copy_rows_add_pos_unpatchify():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(3)
    n, s, sc, c = 2, 16, 5, 24
    L = s + sc
    src = torch.randn(n * sc, 3 * c, generator=g).half()
    J = torch.zeros(n, L, 3 * c, dtype=torch.float16, device=DEV)
    K.copy_rows(src.to(DEV), J[:, s:, :], rows_per_group=sc, group_stride=L)
    ref = torch.zeros(n, L, 3 * c, dtype=torch.float16)
    ref[:, s:] = src.view(n, sc, 3 * c)
    assert torch.equal(J.cpu(), ref)
    x = torch.randn(n, s, c, generator=g).half()
    pos = torch.randn(s, c, generator=g).half()
    assert torch.equal(K.add_pos(x.to(DEV), pos.to(DEV)).cpu(), x + pos)
    b, h, w, p, co = 2, 3, 5, 2, 16
    t = torch.randn(b * h * w, p * p * co, generator=g).half()
    ref = torch.einsum("nhwpqc->nchpwq", t.view(b, h, w, p, p, co)).reshape(b, co, h * p, w * p)
    got = K.unpatchify(t.to(DEV), b, h, w, p, co)
    assert torch.equal(K.nhwc_to_nchw(got).cpu(), ref)


def test_cfg_euler_step_bit_exact():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(4)
    ts, sig = flowmatch_tables(7)
    b = 2
    lat = torch.randn(b, 8, 8, 16, generator=g).half()
    mo = torch.randn(2 * b, 8, 8, 16, generator=g).half()
    ld = lat.to(DEV)
    nxt = torch.empty(2 * b, 8, 8, 16, dtype=torch.float16, device=DEV)
    idx = torch.tensor([3], dtype=torch.int32, device=DEV)
    K.cfg_euler_step(ld, mo.to(DEV), 7.0, sig.to(DEV), idx, nxt)
    ref = euler_step(mo, 3, lat, sig, 7.0)
    assert torch.equal(ld.cpu(), ref)
    assert torch.equal(nxt.cpu(), torch.cat([ref, ref]))
    assert idx.item() == 4


# ------------------------------------------------------------------ model level
@pytest.mark.parametrize("qc", [None,
                                dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
                                dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)])
def test_tiny_mmdit_eval_matches_oracle(qc):
    model = _model()
    cfg = model.pipeline.transformer.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.transformer.state_dict().items()}
    if qc is not None:
        model.quantize(quant_config=dict(qc), quantTransformer=True)
        assert model.quantized_components == ["transformer"]
    x, enc, pooled = _inputs(cfg, 11)
    got = _one_eval(model, x, 987.38, enc, pooled)
    assert torch.isfinite(got).all()
    q = None if qc is None else dict(qc)
    ref = RefMMDiT(_cfgdict(cfg), sd, q).forward(x, 987.38, enc, pooled)
    ref32 = RefMMDiT(_cfgdict(cfg), sd, q, variant="fp32").forward(x, 987.38, enc, pooled)
    _check_parity(got, ref, ref32, f"tiny MMDiT eval {qc}")


def test_sd3_medium_shaped_block_no_qk_norm():
    """qk_norm=None (SD3-Medium style) and 3 blocks, batch 2 (CFG 4), odd context length."""
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    from qdiff.models import StableDiffusion3_5
    from qdiff.pipeline_io import QDiffPipeline
    cfg = tiny_mmdit_config(num_layers=3, qk_norm=None, num_attention_heads=3, caption_projection_dim=192)
    tr = SD3Transformer2DModel(cfg).half().init_synthetic(5).to(DEV)
    sd = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    model = StableDiffusion3_5(QDiffPipeline(transformer=tr, class_name="StableDiffusion3Pipeline"),
                               "StableDiffusion3Pipeline", False, {}, None)
    qc = dict(w_bit=4, a_bit=8, q_group_size=64, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantTransformer=True)
    x, enc, pooled = _inputs(cfg, 12, b=2, sc=77)
    got = _one_eval(model, x, 500.0, enc, pooled)
    ref = RefMMDiT(_cfgdict(cfg), sd, qc).forward(x, 500.0, enc, pooled)
    ref32 = RefMMDiT(_cfgdict(cfg), sd, qc, variant="fp32").forward(x, 500.0, enc, pooled)
    _check_parity(got, ref, ref32, "SD3-M-shaped tiny MMDiT W4A8")


@pytest.mark.timeout(600)
def test_sd35_large_width_two_blocks_512():
    """SD3.5-Large width (C = 2432, 38 heads x 64, RMSNorm qk-norm, joint_attention_dim 4096,
    pooled 2048, pos_embed_max_size 192) with 2 of its 38 blocks, 512^2 latents (S = 1024) and
    the 333-token T5+CLIP context, W4A16 g128, CFG batch 2 - against the fp32 oracle with the
    spread bound of the tiny model (the half CPU oracle is too slow at this width on the box)."""
    import dataclasses as dc
    import time
    from qdiff.mmdit import SD35_LARGE, SD3Transformer2DModel
    from qdiff.models import StableDiffusion3_5
    from qdiff.pipeline_io import QDiffPipeline
    t0 = time.time()
    cfg = dc.replace(SD35_LARGE, num_layers=2, sample_size=64)
    with torch.device(DEV):
        tr = SD3Transformer2DModel(cfg).half()
    tr.init_synthetic(7, rng_device=DEV)
    sd = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    model = StableDiffusion3_5(QDiffPipeline(transformer=tr, class_name="StableDiffusion3Pipeline"),
                               "StableDiffusion3Pipeline", False, {}, None)
    qc = dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False)
    model.quantize(quant_config=dict(qc), quantTransformer=True)
    x, enc, pooled = _inputs(cfg, 13, b=1, sc=333)
    got = _one_eval(model, x, 974.1, enc, pooled)
    torch.cuda.synchronize()
    print(f"[sd35-width] gpu eval {time.time() - t0:.1f}s", flush=True)
    ref32 = RefMMDiT(_cfgdict(cfg), sd, qc, variant="fp32").forward(x, 974.1, enc, pooled)
    print(f"[sd35-width] fp32 oracle {time.time() - t0:.1f}s", flush=True)
    mx32, mean32 = _rel_errs(got, ref32)
    print(f"SD3.5-L width, 2 blocks, W4A16: gpu-vs-fp32 max {mx32:.4g} mean {mean32:.4g}")
    assert torch.isfinite(got).all()
    assert mx32 <= 0.02 and mean32 <= 0.004, (mx32, mean32)


@pytest.mark.parametrize("qc", [None,
                                dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
                                dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)])
def test_tiny_mmdit_x_eval_matches_oracle(qc):
    """SD3.5-Medium-shaped MMDiT-X (dual attention in blocks 0-1 of 3: SD35AdaLayerNormZeroX's
    9C adaLN, image-only attn2 with RMSNorm qk-norm) vs the oracle, CFG batch 2, odd context."""
    model = _model("synthetic:sd35m-tiny", seed=2)
    tr = model.pipeline.transformer
    cfg = tr.config
    assert tr.transformer_blocks[0].attn2 is not None and tr.transformer_blocks[2].attn2 is None
    sd = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    if qc is not None:
        model.quantize(quant_config=dict(qc), quantTransformer=True)
    x, enc, pooled = _inputs(cfg, 21, b=2, sc=37)
    got = _one_eval(model, x, 641.5, enc, pooled)
    assert torch.isfinite(got).all()
    q = None if qc is None else dict(qc)
    ref = RefMMDiT(_cfgdict(cfg), sd, q).forward(x, 641.5, enc, pooled)
    ref32 = RefMMDiT(_cfgdict(cfg), sd, q, variant="fp32").forward(x, 641.5, enc, pooled)
    _check_parity(got, ref, ref32, f"tiny MMDiT-X eval {qc}")


@pytest.mark.timeout(600)
def test_sd35_medium_width_dual_blocks_512():
    """SD3.5-Medium width (C = 1536, 24 heads x 64, pos_embed_max_size 384) with 2 of its
    blocks, both MMDiT-X (dual attention), 512^2 latents, 333-token context, W4A16 g128,
    CFG batch 2, against the fp32 oracle (bound of the SD3.5-L width case)."""
    import dataclasses as dc
    from qdiff.mmdit import SD35_MEDIUM, SD3Transformer2DModel
    from qdiff.models import StableDiffusion3_5
    from qdiff.pipeline_io import QDiffPipeline
    cfg = dc.replace(SD35_MEDIUM, num_layers=2, sample_size=64, dual_attention_layers=(0, 1))
    with torch.device(DEV):
        tr = SD3Transformer2DModel(cfg).half()
    tr.init_synthetic(9, rng_device=DEV)
    sd = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    model = StableDiffusion3_5(QDiffPipeline(transformer=tr, class_name="StableDiffusion3Pipeline"),
                               "StableDiffusion3Pipeline", False, {}, None)
    qc = dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False)
    model.quantize(quant_config=dict(qc), quantTransformer=True)
    x, enc, pooled = _inputs(cfg, 14, b=1, sc=333)
    got = _one_eval(model, x, 811.0, enc, pooled)
    ref32 = RefMMDiT(_cfgdict(cfg), sd, qc, variant="fp32").forward(x, 811.0, enc, pooled)
    mx32, mean32 = _rel_errs(got, ref32)
    print(f"SD3.5-M width, 2 dual blocks, W4A16: gpu-vs-fp32 max {mx32:.4g} mean {mean32:.4g}")
    assert torch.isfinite(got).all()
    assert mx32 <= 0.02 and mean32 <= 0.004, (mx32, mean32)


def test_quantized_buffers_bit_exact_and_output_quant_names():
    from oracle.unet_ref import quantize_state_dict
    from qdiff.fake_quant import WxAxLinear
    model = _model(seed=1)
    tr = model.pipeline.transformer
    sd = {k: v.detach().cpu() for k, v in tr.state_dict().items()}
    qc = dict(w_bit=4, a_bit=8, q_group_size=128, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantTransformer=True)
    qsd, flags = quantize_state_dict(sd, qc)
    got = tr.state_dict()
    assert set(got) == set(sd)
    for k, v in qsd.items():
        assert torch.equal(got[k].cpu().view(torch.int16), v.view(torch.int16)), k
    oq = sorted(n for n, m in tr.named_modules() if isinstance(m, WxAxLinear) and m.output_quant_name != "None")
    assert oq == sorted(f"transformer_blocks.{i}.attn.add_{p}_proj" for i in range(2) for p in "qkv")


def test_flowmatch_graph_replay_equals_eager_and_oracle_denoise():
    model = _model(seed=2)
    cfg = model.pipeline.transformer.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.transformer.state_dict().items()}
    qc = dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False)
    model.quantize(quant_config=dict(qc), quantTransformer=True)
    g = torch.Generator().manual_seed(42)
    lat = torch.randn(1, 16, cfg.sample_size, cfg.sample_size, generator=g).half()
    pe = torch.randn(1, 40, cfg.joint_attention_dim, generator=g).half()
    ne = torch.randn(1, 40, cfg.joint_attention_dim, generator=g).half()
    pp = torch.randn(1, cfg.pooled_projection_dim, generator=g).half()
    npp = torch.randn(1, cfg.pooled_projection_dim, generator=g).half()
    hw = cfg.sample_size * 8
    kw = dict(prompt_embeds=pe, negative_prompt_embeds=ne, pooled_prompt_embeds=pp, negative_pooled_prompt_embeds=npp,
              lat=lat, height=hw, width=hw, num_inference_steps=4, output_type="latent")
    eager = model.generate(use_graph=False, **kw).cpu()
    graph = model.generate(use_graph=True, **kw).cpu()
    graph2 = model.generate(use_graph=True, **kw).cpu()
    assert torch.equal(graph, graph2)
    assert torch.equal(eager, graph)
    ts, sig = flowmatch_tables(4)
    enc, pooled = torch.cat([ne, pe]), torch.cat([npp, pp])
    ref = denoise(RefMMDiT(_cfgdict(cfg), sd, qc), lat, enc, pooled, ts, sig, 7.0)
    ref32 = denoise(RefMMDiT(_cfgdict(cfg), sd, qc, variant="fp32"), lat, enc, pooled, ts, sig, 7.0)
    _check_parity(graph, ref, ref32, "tiny MMDiT W4A16 4-step flow-match denoise")


def test_awq_facade_save_load_roundtrip(tmp_path):
    from qdiff.models import AWQ, StableDiffusion3_5
    model = AWQ.from_pretrained("synthetic:sd35-tiny", device=DEV, seed=3)
    assert isinstance(model, StableDiffusion3_5)
    with pytest.raises(Exception):
        model.get_model_layers_unet()
    model.quantize(quant_config=dict(w_bit=4, a_bit=8, q_group_size=128, quantize_act=True), quantTransformer=True)
    model.save_quantized(str(tmp_path))
    re = StableDiffusion3_5.from_quantized(str(tmp_path), "StableDiffusion3Pipeline")
    a, b = model.pipeline.transformer.state_dict(), re.pipeline.transformer.state_dict()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    cfg = model.pipeline.transformer.config
    x, enc, pooled = _inputs(cfg, 4)
    assert torch.equal(_one_eval(model, x, 501.0, enc, pooled), _one_eval(re, x, 501.0, enc, pooled))
    out = model.generate(prompt=["a red cube"], height=cfg.sample_size * 8, width=cfg.sample_size * 8,
                         num_inference_steps=2, output_type="latent")
    assert out.shape == (1, 16, cfg.sample_size, cfg.sample_size) and torch.isfinite(out.float()).all()
