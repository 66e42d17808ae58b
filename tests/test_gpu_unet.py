"""End-to-end parity of the fused GPU UNet / denoising loop with the CPU oracle
(oracle/unet_ref.py: golden-pinned fake-quant math + torch-CPU fp16 diffusers ops).

Tolerance (stated once, used below): the GPU path differs from the CPU oracle only by fp32
accumulation order inside GEMMs / norms / attention, i.e. by <= ~1 fp16 ulp per op; a 1-ulp
shift can move a value across a fake-quant rounding boundary (one quantization step, 1/127 of
the channel amax at 8 bits).  Over a whole UNet these stay small relative to the output
scale: we require max|gpu - cpu| <= 3e-2 * max|cpu| and mean|gpu - cpu| <= 2e-3 * max|cpu| for
one UNet evaluation, and 5e-2 / 5e-3 after several denoising steps.
"""
import dataclasses

import pytest
import torch

from oracle.unet_ref import RefUNet, denoise

pytestmark = pytest.mark.gpu


def _cfgdict(cfg):
    return {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}


def _rel_errs(got, ref):
    got, ref = got.float().cpu(), ref.float().cpu()
    scale = ref.abs().max().item()
    d = (got - ref).abs()
    return d.max().item() / scale, d.mean().item() / scale


def _model(name="synthetic:tiny", seed=0):
    from qdiff.models import StableDiffusion1_x
    return StableDiffusion1_x.from_pretrained(name, device="cuda:0", seed=seed)


def _one_eval(model, x, t, ctx):
    """One UNet evaluation through the fused NHWC path."""
    from qdiff import kernels as K
    from qdiff.scheduler import ddim_tables
    unet = model.pipeline.unet
    dev = torch.device("cuda:0")
    kv = unet.prepare_context(ctx.to(dev))
    xh = K.nchw_to_nhwc(x.to(dev), 8)
    ts = torch.tensor([float(t)], device=dev)
    temb = K.timestep_embedding(ts, None, x.shape[0], unet.config.block_out_channels[0])
    out = unet.fwd(xh, temb, kv)
    return K.nhwc_to_nchw(out, 4).cpu()


@pytest.mark.parametrize("qc", [None,
                                dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True),
                                dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
                                dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True,
                                     weight_quant_type="per_channel")])
def test_tiny_unet_eval_matches_oracle(qc):
    model = _model()
    cfg = model.pipeline.unet.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.unet.state_dict().items()}
    if qc is not None:
        model.quantize(quant_config=dict(qc), quantUnet=True)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    ctx = torch.randn(2, 77, cfg.cross_attention_dim, generator=g).half()
    got = _one_eval(model, x, 981, ctx)
    ref = RefUNet(_cfgdict(cfg), sd, None if qc is None else dict(qc)).forward(x, 981, ctx)
    mx, mean = _rel_errs(got, ref)
    assert mx <= 3e-2 and mean <= 2e-3, (mx, mean)


def test_quantized_buffers_bit_exact():
    """After quantize(), every WxAx buffer equals the oracle's quantization of the same weights."""
    from oracle.unet_ref import quantize_state_dict
    model = _model()
    sd = {k: v.detach().cpu() for k, v in model.pipeline.unet.state_dict().items()}
    qc = dict(w_bit=4, a_bit=8, q_group_size=128, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantUnet=True)
    qsd, flags = quantize_state_dict(sd, qc)
    got = model.pipeline.unet.state_dict()
    assert set(got) == set(sd)
    for k, v in qsd.items():
        assert torch.equal(got[k].cpu().view(torch.int16), v.view(torch.int16)), k
    assert model.quantized_components == ["unet"]


def test_graph_replay_equals_eager_and_oracle_denoise():
    from qdiff.scheduler import ddim_tables
    model = _model(seed=1)
    cfg = model.pipeline.unet.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.unet.state_dict().items()}
    qc = dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantUnet=True)
    g = torch.Generator().manual_seed(42)
    lat = torch.randn(2, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    pe = torch.randn(2, 77, cfg.cross_attention_dim, generator=g).half()
    ne = torch.randn(2, 77, cfg.cross_attention_dim, generator=g).half()
    hw = cfg.sample_size * 8
    kw = dict(prompt_embeds=pe, negative_prompt_embeds=ne, lat=lat, height=hw, width=hw, num_inference_steps=4,
              output_type="latent")
    eager = model.generate(use_graph=False, **kw).cpu()
    graph = model.generate(use_graph=True, **kw).cpu()
    graph2 = model.generate(use_graph=True, **kw).cpu()   # replay of the cached graph
    assert torch.equal(eager, graph) and torch.equal(graph, graph2)
    ts, a_t, a_p = ddim_tables(4)
    ref = denoise(RefUNet(_cfgdict(cfg), sd, qc), lat, torch.cat([ne, pe]), ts, a_t, a_p, 7.5)
    mx, mean = _rel_errs(graph, ref)
    assert mx <= 5e-2 and mean <= 5e-3, (mx, mean)


def test_sq_quantize_fold_matches_oracle_fold():
    """SmoothQuant: the device fold of the calibrated means equals the oracle fold (bit-exact up
    to rare 1-ulp pow differences), and the swap follows."""
    import numpy as np
    from oracle import fake_quant_np as FQ
    from qdiff.fake_quant import WxAxLinear
    model = _model(seed=2)
    unet = model.pipeline.unet
    blocks = model.get_smoothing_blocks()
    before = {n: (b.norm1.weight.detach().cpu().clone(), [l.weight.detach().cpu().clone() for l in
                  (b.attn1.to_q, b.attn1.to_k, b.attn1.to_v)]) for n, b in blocks.items()}
    captured = {}
    from qdiff import quantizer as Q
    orig = Q.SqQuantizer.smooth_ln_fcs

    def spy(self, ln, fcs, act, model_type="transformers", alpha=0.5):
        captured.setdefault(id(ln), act.detach().cpu().clone())
        return orig(self, ln, fcs, act, model_type, alpha)

    Q.SqQuantizer.smooth_ln_fcs = spy
    try:
        model.quantize(quant_config=dict(w_bit=8, a_bit=8, quantize_act=True), quantType="sq", quantUnet=True,
                       calibration=dict(n_samples=2, batch_size=2, num_inference_steps=2))
    finally:
        Q.SqQuantizer.smooth_ln_fcs = orig
    assert sum(isinstance(m, WxAxLinear) for m in unet.modules()) > 0
    for n, b in blocks.items():
        act = captured[id(b.norm1)].numpy()
        lw0, ws0 = before[n]
        sc = FQ.smooth_scales(act, [w.numpy() for w in ws0], 0.8)
        lw_ref = (lw0.numpy().astype(np.float32) / sc.astype(np.float32)).astype(np.float16)
        nbad = int((b.norm1.weight.detach().cpu().numpy() != lw_ref).sum())
        assert nbad <= 2, (n, nbad)


def test_save_load_quantized_roundtrip(tmp_path):
    from qdiff.models import StableDiffusion1_x
    model = _model(seed=3)
    model.quantize(quant_config=dict(w_bit=4, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    model.save_quantized(str(tmp_path))
    assert (tmp_path / "quant_components.json").exists()
    re = StableDiffusion1_x.from_quantized(str(tmp_path), "StableDiffusionPipeline")
    a = model.pipeline.unet.state_dict()
    b = re.pipeline.unet.state_dict()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    cfg = model.pipeline.unet.config
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    ctx = torch.randn(2, 77, cfg.cross_attention_dim, generator=g).half()
    assert torch.equal(_one_eval(model, x, 501, ctx), _one_eval(re, x, 501, ctx))


def test_sd15_full_unet_eval_matches_oracle():
    """One full-size SD1.5 (859.5 M params) W8A8 UNet evaluation at 64x64 latents, batch 2."""
    model = _model("synthetic:sd15", seed=0)
    cfg = model.pipeline.unet.config
    sd = {k: v.detach().cpu() for k, v in model.pipeline.unet.state_dict().items()}
    qc = dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantUnet=True)
    g = torch.Generator().manual_seed(42)
    x = torch.randn(2, 4, 64, 64, generator=g).half()
    ctx = torch.randn(2, 77, 768, generator=g).half()
    got = _one_eval(model, x, 981, ctx)
    ref = RefUNet(_cfgdict(cfg), sd, qc).forward(x, 981, ctx)
    mx, mean = _rel_errs(got, ref)
    print(f"SD1.5 W8A8 one eval: max rel {mx:.3g}, mean rel {mean:.3g}")
    assert mx <= 3e-2 and mean <= 2e-3, (mx, mean)
