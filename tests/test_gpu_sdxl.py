"""SDXL (config C4) on the GPU vs the CPU oracle: the "text_time" additional conditioning,
linear proj_in / proj_out, multi-layer transformer stacks, and diffusers' EulerDiscreteScheduler
loop (init_noise_sigma, scale_model_input, Euler step).  Same self-calibrated tolerance as
tests/test_gpu_unet.py; the CFG + Euler step kernel is bit-exact to the oracle's torch-CPU ops."""
import dataclasses

import pytest
import torch

from oracle.unet_ref import RefUNet, denoise_euler, euler_step, euler_tables

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


def _model(seed=0):
    from qdiff.models import StableDiffusionXL
    return StableDiffusionXL.from_pretrained("synthetic:sdxl-tiny", device=DEV, seed=seed)


def _cond(cfg, seed, b=1):
    g = torch.Generator().manual_seed(seed)
    pooled = cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim
    x = torch.randn(2 * b, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    ctx = torch.randn(2 * b, 77, cfg.cross_attention_dim, generator=g).half()
    text = torch.randn(2 * b, pooled, generator=g).half()
    hw = cfg.sample_size * 8
    time_ids = torch.tensor([[hw, hw, 0, 0, hw, hw]] * (2 * b), dtype=torch.float32)
    return x, ctx, text, time_ids


def _one_eval(model, x, t, ctx, text, time_ids):
    from qdiff import kernels as K
    unet = model.pipeline.unet
    cfg = unet.config
    kv = unet.prepare_context(ctx.to(DEV))
    xh = K.nchw_to_nhwc(x.to(DEV), 8)
    temb = K.timestep_embedding(torch.tensor([float(t)], device=DEV), None, x.shape[0], cfg.block_out_channels[0])
    tid = time_ids.to(DEV).reshape(-1).contiguous()
    te = K.timestep_embedding(tid, None, tid.numel(), cfg.addition_time_embed_dim, per_row=True)
    add = K.concat_c(text.to(DEV).contiguous(), te.view(x.shape[0], -1))
    return K.nhwc_to_nchw(unet.fwd(xh, temb, kv, add_emb_in=add), 4).cpu()


@pytest.mark.parametrize("qc", [None, dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True),
                                dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False)])
def test_tiny_sdxl_eval_matches_oracle(qc):
    model = _model()
    cfg = model.pipeline.unet.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.unet.state_dict().items()}
    if qc is not None:
        model.quantize(quant_config=dict(qc), quantUnet=True)
    x, ctx, text, tid = _cond(cfg, 21)
    got = _one_eval(model, x, 961.0, ctx, text, tid)
    q = None if qc is None else dict(qc)
    ref_m = RefUNet(_cfgdict(cfg), sd, q)
    add = ref_m.add_embeds(text, tid)
    ref = ref_m.forward(x, 961.0, ctx, add)
    ref32 = RefUNet(_cfgdict(cfg), sd, q, variant="fp32").forward(x, 961.0, ctx, add)
    _check_parity(got, ref, ref32, f"tiny SDXL eval {qc}")


def test_euler_discrete_step_and_scaling_bit_exact():
    from qdiff import kernels as K
    from qdiff.scheduler import euler_discrete_tables
    ts, sig, dsc, init = euler_discrete_tables(10)
    ots, osig, oinit = euler_tables(10)
    assert torch.equal(ts, ots) and torch.equal(sig, osig) and init.item() == oinit.item()
    g = torch.Generator().manual_seed(5)
    b = 2
    lat = torch.randn(b, 4, 8, 8, generator=g).half()
    mo = torch.randn(2 * b, 4, 8, 8, generator=g).half()
    ld = K.nchw_to_nhwc(lat.to(DEV), 8)
    nxt = torch.zeros(2 * b, 8, 8, 8, dtype=torch.float16, device=DEV)
    idx = torch.tensor([3], dtype=torch.int32, device=DEV)
    K.cfg_euler_discrete_step(ld, K.nchw_to_nhwc(mo.to(DEV), 8), 5.0, sig.to(DEV), dsc.to(DEV), idx, nxt, c=4)
    ref = euler_step(mo, 3, lat, osig, 5.0)
    assert torch.equal(K.nhwc_to_nchw(ld, 4).cpu(), ref)
    refin = torch.cat([ref] * 2) / ((osig[4] ** 2 + 1) ** 0.5)
    assert torch.equal(K.nhwc_to_nchw(nxt, 4).cpu(), refin)
    assert idx.item() == 4
    # prepare_latents * init_noise_sigma, then the first scale_model_input
    l0 = K.nchw_to_nhwc(lat.to(DEV), 8)
    n0 = torch.zeros(2 * b, 8, 8, 8, dtype=torch.float16, device=DEV)
    K.scale_latents(l0, float(oinit), float(dsc[0]), next_in=n0, c=4)
    r0 = lat * oinit
    assert torch.equal(K.nhwc_to_nchw(l0, 4).cpu(), r0)
    assert torch.equal(K.nhwc_to_nchw(n0, 4).cpu(), torch.cat([r0] * 2) / ((osig[0] ** 2 + 1) ** 0.5))


def test_sdxl_euler_graph_denoise_matches_oracle():
    model = _model(seed=1)
    cfg = model.pipeline.unet.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.unet.state_dict().items()}
    qc = dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantUnet=True)
    g = torch.Generator().manual_seed(43)
    pooled = cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim
    lat = torch.randn(1, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    pe = torch.randn(1, 77, cfg.cross_attention_dim, generator=g).half()
    ne = torch.randn(1, 77, cfg.cross_attention_dim, generator=g).half()
    pp = torch.randn(1, pooled, generator=g).half()
    npp = torch.randn(1, pooled, generator=g).half()
    hw = cfg.sample_size * 8
    kw = dict(prompt_embeds=pe, negative_prompt_embeds=ne, pooled_prompt_embeds=pp, negative_pooled_prompt_embeds=npp,
              lat=lat, height=hw, width=hw, num_inference_steps=4, output_type="latent")
    eager = model.generate(use_graph=False, **kw).cpu()
    graph = model.generate(use_graph=True, **kw).cpu()
    assert torch.equal(eager, graph)
    assert torch.equal(graph, model.generate(use_graph=True, **kw).cpu())
    ts, sig, init = euler_tables(4)
    ctx = torch.cat([ne, pe])
    tid = torch.tensor([[hw, hw, 0, 0, hw, hw]] * 2, dtype=torch.float32)
    r16, r32 = RefUNet(_cfgdict(cfg), sd, qc), RefUNet(_cfgdict(cfg), sd, qc, variant="fp32")
    add = r16.add_embeds(torch.cat([npp, pp]), tid)
    ref = denoise_euler(r16, lat, ctx, add, ts, sig, init, 5.0)
    ref32 = denoise_euler(r32, lat, ctx, add, ts, sig, init, 5.0)
    _check_parity(graph, ref, ref32, "tiny SDXL W8A8 4-step Euler denoise")


def test_sdxl_adapter_surface_and_prompt_generate():
    from qdiff.models import AWQ, StableDiffusionXL
    model = AWQ.from_pretrained("synthetic:sdxl-tiny", device=DEV, seed=2)
    assert isinstance(model, StableDiffusionXL)
    with pytest.raises(Exception):
        model.checkQuantStatus(quantTransformer=True)
    model.quantize(quant_config=dict(w_bit=4, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    cfg = model.pipeline.unet.config
    out = model.generate(prompt=["a red cube", "a blue ball"], height=cfg.sample_size * 8, width=cfg.sample_size * 8,
                         num_inference_steps=3, output_type="latent")
    assert out.shape == (2, 4, cfg.sample_size, cfg.sample_size) and torch.isfinite(out.float()).all()
