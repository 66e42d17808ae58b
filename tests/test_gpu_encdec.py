"""Text encoder (CLIP) and VAE decoder on the GPU against their oracles.

CLIP: transformers' own CLIPTextModel / CLIPTextModelWithProjection (the library the reference's
pipelines run; version pinned by the image) loaded with the same weights, on the CPU in fp32 and
in fp16.  VAE: oracle/vae_ref.py (diffusers' decoder restated; diffusers itself is absent).
Criterion: the self-calibrated rule of tests/test_gpu_unet.py (within 1.5 x the oracle's own
half-vs-fp32 spread + 2e-3 of both variants, max and mean relative to max|ref|); kernels with a
single rounding (embedding add, activations, postprocess) bit-exact or within 1 fp16 ulp.
"""
import dataclasses

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel_errs(got, ref):
    got, ref = got.float().cpu(), ref.float().cpu()
    scale = ref.abs().max().item()
    d = (got - ref).abs()
    return d.max().item() / scale, d.mean().item() / scale


def _check_parity(got, ref, ref32, what, floor=2e-3):
    smx, smean = _rel_errs(ref32, ref)
    mx, mean = _rel_errs(got, ref)
    mx32, mean32 = _rel_errs(got, ref32)
    print(f"{what}: gpu-vs-half max {mx:.4g} mean {mean:.4g} | gpu-vs-fp32 max {mx32:.4g} mean {mean32:.4g} | "
          f"oracle spread max {smx:.4g} mean {smean:.4g}", flush=True)
    tmx, tmean = 1.5 * smx + floor, 1.5 * smean + floor
    assert mx <= tmx and mean <= tmean, (mx, mean, tmx, tmean)
    assert mx32 <= tmx and mean32 <= tmean, (mx32, mean32, tmx, tmean)


# ------------------------------------------------------------------ kernels
@pytest.mark.parametrize("b,heads,s,d", [(2, 12, 77, 64), (3, 2, 77, 32), (1, 20, 77, 64), (2, 1, 130, 40)])
def test_attention_causal(b, heads, s, d):
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(s + d)
    q, k, v = ((torch.randn(b, s, heads * d, generator=g) * 2).half() for _ in range(3))
    got = K.attention_causal(q.to(DEV), k.to(DEV), v.to(DEV), heads).cpu()
    hv = lambda t: t.float().view(b, s, heads, d).transpose(1, 2)
    ref = F.scaled_dot_product_attention(hv(q), hv(k), hv(v), is_causal=True).transpose(1, 2).reshape(b, s, -1)
    err = (got.float() - ref).abs()
    assert err.max().item() <= 4e-3 * max(1.0, ref.abs().max().item()), err.max().item()


@pytest.mark.parametrize("s,d", [(4096, 512), (1024, 512), (256, 320)])
def test_attention_wide_head(s, d):
    """the VAE mid block's single head (512 channels at 64x64 latents) and a 320-wide one."""
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(s)
    b = 1
    q, k, v = (torch.randn(b, s, d, generator=g).half() for _ in range(3))
    got = K.attention(q.to(DEV), k.to(DEV), v.to(DEV), 1).cpu()
    ref = F.scaled_dot_product_attention(q.float()[:, None], k.float()[:, None], v.float()[:, None])[:, 0]
    err = (got.float() - ref).abs()
    assert err.max().item() <= 4e-3 * max(1.0, ref.abs().max().item()), err.max().item()


def test_embed_act_gather_postprocess_bit_exact():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(3)
    tok = (torch.randn(1000, 64, generator=g) * 0.02).half()
    pos = (torch.randn(77, 64, generator=g) * 0.02).half()
    ids = torch.randint(0, 1000, (3, 77), generator=g)
    got = K.embed_tokens(ids.to(DEV), tok.to(DEV), pos.to(DEV)).cpu()
    assert torch.equal(got, (tok[ids] + pos[None]).view(-1, 64))
    x = (torch.randn(4096, generator=g) * 4).half()
    for kind, ref in (("quick_gelu", x * torch.sigmoid(1.702 * x)), ("gelu", F.gelu(x.float()).half())):
        got = K.clip_act(x.to(DEV), kind).cpu()
        ulp = torch.clamp(ref.float().abs(), min=2.0 ** -14) * 2.0 ** -10
        # quick_gelu: a 1-ulp step of the fp16 sigmoid (subnormal where x << 0) moves x * s by |x| ulp(s)
        sig = torch.sigmoid(1.702 * x).float()
        ulp_s = torch.clamp(sig.abs(), min=2.0 ** -14) * 2.0 ** -10 if kind == "quick_gelu" else 0 * sig
        d = (got.float() - ref.float()).abs()
        # gelu: for x < -3 the CPU's and this kernel's f32 1 + erf(x / sqrt 2) both cancel (erfc ~ 1e-4
        # from two ~1-ulp erf values), so the tiny results agree to ~1e-3 relative, not to the fp16 ulp
        tail = 1e-6 if kind == "gelu" else 1e-7
        bad = d > ulp + x.float().abs() * ulp_s + tail
        # the exact-erf GELU's branch-free erfc fit (common.h gelu_f) differs from libm's erf by an
        # fp16 ulp on a few % of inputs; quick_gelu is exact on > 99 %
        assert not bad.any() and (d == 0).float().mean() > (0.99 if kind == "quick_gelu" else 0.9), \
            (kind, int((d > 0).sum()), x[bad][:8].tolist(), got[bad][:8].tolist(), ref[bad][:8].tolist())
    rows = torch.randn(3 * 77, 64, generator=g).half()
    idx = torch.tensor([5, 77 + 76, 154], dtype=torch.int64)
    assert torch.equal(K.gather_rows(rows.to(DEV), idx.to(DEV)).cpu(), rows[idx])
    y = (torch.randn(2, 16, 24, 8, generator=g) * 1.5).half()
    a, u = K.vae_postprocess(y.to(DEV), 3, want_nchw=True, want_u8=True)
    refimg = (y[..., :3].permute(0, 3, 1, 2) / 2 + 0.5).clamp(0, 1)
    assert torch.equal(a.cpu(), refimg)
    from oracle.vae_ref import to_uint8
    assert np.array_equal(u.cpu().numpy(), to_uint8(refimg))
    lat = torch.randn(2, 8, 8, 16, generator=g).half()
    z = K.vae_prescale(lat.to(DEV), 16, 1.5305, 0.0609, cout_pad=16).cpu()
    assert torch.equal(z, lat / 1.5305 + 0.0609)
    z = K.vae_prescale(lat[..., :8].contiguous().to(DEV), 4, 0.18215, None, cout_pad=8).cpu()
    assert torch.equal(z[..., :4], lat[..., :4] / 0.18215) and not z[..., 4:].any()


# ------------------------------------------------------------------ CLIP text encoder
def _hf_clip(cfg, sd, dtype):
    from transformers import CLIPTextConfig as HC
    from transformers import CLIPTextModel as HM
    from transformers import CLIPTextModelWithProjection as HP
    m = (HP if cfg.projection_dim else HM)(HC(**cfg.to_transformers()))
    if cfg.projection_dim is None:
        sd = {k[len("text_model."):]: v for k, v in sd.items()}
    missing, unexpected = m.load_state_dict({k: v.float() for k, v in sd.items()}, strict=False)
    assert not [k for k in missing if "position_ids" not in k], missing
    return m.to(dtype).eval()


def _hf_outputs(m, ids, cfg, hidden_state, pooled):
    with torch.no_grad():
        o = m(input_ids=ids, output_hidden_states=True)
    h = o.last_hidden_state if hidden_state == -1 else o.hidden_states[hidden_state]
    p = None
    if pooled:
        p = o.text_embeds if cfg.projection_dim else o.pooler_output
    return h, p


@pytest.mark.parametrize("which", ["tiny", "tiny_g", "clip_l", "clip_l_proj"])
def test_clip_text_encoder_matches_transformers(which):
    from qdiff.clip import CLIP_L, CLIP_L_PROJ, CLIPTextModel, HashTokenizer, tiny_clip_config
    cfg = {"tiny": tiny_clip_config(), "tiny_g": tiny_clip_config(hidden=96, heads=3, layers=3, projection_dim=48,
                                                                   act="gelu"),
           "clip_l": CLIP_L, "clip_l_proj": CLIP_L_PROJ}[which]
    m = CLIPTextModel(cfg).half().init_synthetic(11)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    tok = HashTokenizer(pad_id=0 if cfg.projection_dim else 49407)
    ids = tok(["a photograph of an astronaut riding a horse", "", "red cube on a blue ball " * 20])
    hs, pooled = (-1, False) if cfg.projection_dim is None else (-2, True)
    got_h, got_p = m.encode(ids, hidden_state=hs, pooled=pooled)
    rh, rp = _hf_outputs(_hf_clip(cfg, sd, torch.float16), ids, cfg, hs, pooled)
    rh32, rp32 = _hf_outputs(_hf_clip(cfg, sd, torch.float32), ids, cfg, hs, pooled)
    _check_parity(got_h, rh, rh32, f"CLIP {which} hidden_states[{hs}]")
    if pooled:
        _check_parity(got_p, rp, rp32, f"CLIP {which} pooled / text_embeds")
    if which in ("tiny", "clip_l"):  # last hidden state AND penultimate from one model
        got_pen, _ = m.encode(ids, hidden_state=-2)
        rpen, _ = _hf_outputs(_hf_clip(cfg, sd, torch.float16), ids, cfg, -2, False)
        rpen32, _ = _hf_outputs(_hf_clip(cfg, sd, torch.float32), ids, cfg, -2, False)
        _check_parity(got_pen, rpen, rpen32, f"CLIP {which} hidden_states[-2]")


# ------------------------------------------------------------------ VAE decoder
def _vae_cfgdict(cfg):
    return {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}


@pytest.mark.parametrize("lat_ch,qc", [(4, None), (16, None),
                                       (4, dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True))])
def test_tiny_vae_decode_matches_oracle(lat_ch, qc):
    from oracle.vae_ref import RefVAEDecoder, postprocess
    from qdiff import kernels as K
    from qdiff.vae import AutoencoderKL, tiny_vae_config
    cfg = tiny_vae_config(lat_ch)
    vae = AutoencoderKL(cfg).half().init_synthetic(5)
    sd = {k: v.clone() for k, v in vae.state_dict().items()}
    vae = vae.to(DEV)
    if qc is not None:
        from qdiff.models import StableDiffusion1_x
        model = StableDiffusion1_x.from_pretrained("synthetic:tiny", device=DEV, seed=0)
        model.pipeline.vae = vae
        model.quantize(quant_config=dict(qc), quantUnet=False, quantVAE=True)
        assert "vae" in model.quantized_components
    g = torch.Generator().manual_seed(7)
    lat = torch.randn(2, lat_ch, 16, 24, generator=g).half()
    y = vae.decode_nhwc(K.nchw_to_nhwc(lat.to(DEV), (lat_ch + 7) // 8 * 8))
    got = K.nhwc_to_nchw(y, 3).cpu()
    ref = RefVAEDecoder(_vae_cfgdict(cfg), sd, qc).decode(lat)
    ref32 = RefVAEDecoder(_vae_cfgdict(cfg), sd, qc, variant="fp32").decode(lat)
    _check_parity(got, ref, ref32, f"tiny VAE decode (latent {lat_ch} ch, {qc})")
    img = vae.decode_images(K.nchw_to_nhwc(lat.to(DEV), (lat_ch + 7) // 8 * 8), "pt").cpu()
    assert torch.equal(img, postprocess(got))


@pytest.mark.timeout(600)
def test_sd_vae_full_size_decode_512():
    """The SD1.x VAE decoder (83.7 M decoder params, 128..512 channels) on 64x64 latents -> 512^2,
    batch 1, against the fp32 oracle (the half oracle's Half conv is scalar on the GPU box's host;
    its spread is taken from the tiny model: bound 0.02 max / 0.004 mean relative)."""
    import time
    from oracle.vae_ref import RefVAEDecoder
    from qdiff import kernels as K
    from qdiff.vae import SD_VAE, AutoencoderKL
    t0 = time.time()
    vae = AutoencoderKL(SD_VAE).half().init_synthetic(3)
    sd = {k: v.clone() for k, v in vae.state_dict().items()}
    vae = vae.to(DEV)
    g = torch.Generator().manual_seed(8)
    lat = torch.randn(1, 4, 64, 64, generator=g).half()
    y = vae.decode_nhwc(K.nchw_to_nhwc(lat.to(DEV), 8))
    got = K.nhwc_to_nchw(y, 3).cpu()
    torch.cuda.synchronize()
    print(f"[vae] gpu decode {time.time() - t0:.1f}s", flush=True)
    ref32 = RefVAEDecoder(_vae_cfgdict(SD_VAE), sd, None, variant="fp32").decode(lat)
    print(f"[vae] fp32 oracle {time.time() - t0:.1f}s", flush=True)
    mx, mean = _rel_errs(got, ref32)
    print(f"SD VAE 512^2 decode: gpu-vs-fp32 max {mx:.4g} mean {mean:.4g}", flush=True)
    assert torch.isfinite(got.float()).all()
    assert mx <= 0.02 and mean <= 0.004, (mx, mean)


# ------------------------------------------------------------------ end to end
def test_tiny_sd15_prompt_to_image_matches_oracle_chain():
    """prompt -> CLIP (GPU) -> 3 DDIM steps (GPU) -> VAE (GPU) -> uint8 image, against
    transformers' CLIP + the UNet oracle loop + the VAE oracle on the same weights."""
    from oracle.unet_ref import RefUNet, ddim_tables, denoise
    from oracle.vae_ref import RefVAEDecoder, postprocess
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:tiny", device=DEV, seed=4)
    pipe = model.pipeline
    unet_cfg = pipe.unet.config
    usd = {k: v.detach().cpu() for k, v in pipe.unet.state_dict().items()}
    tsd = {k: v.detach().cpu() for k, v in pipe.text_encoder.state_dict().items()}
    vsd = {k: v.detach().cpu() for k, v in pipe.vae.state_dict().items()}
    g = torch.Generator().manual_seed(9)
    hw = unet_cfg.sample_size * 8
    lat = torch.randn(2, 4, unet_cfg.sample_size, unet_cfg.sample_size, generator=g).half()
    prompts = ["a red cube", "a watercolor fox in the snow"]
    kw = dict(prompt=prompts, lat=lat, height=hw, width=hw, num_inference_steps=3)
    pt = model.generate(output_type="pt", **kw).cpu()
    npimg = model.generate(**kw)
    pil = model.generate(output_type="pil", **kw)
    lat_out = model.generate(output_type="latent", **kw).cpu()
    assert pt.shape == (2, 3, hw, hw) and pt.dtype == torch.float16
    assert isinstance(npimg, np.ndarray) and npimg.shape == (2, hw, hw, 3) and npimg.dtype == np.float32
    assert np.array_equal(npimg, pt.permute(0, 2, 3, 1).float().numpy())
    assert len(pil) == 2 and pil[0].size == (hw, hw)
    # oracle chain
    tcfg = pipe.text_encoder.config
    ids = pipe.tokenizer(prompts)
    nids = pipe.tokenizer([""] * 2)
    from qdiff import vae as V
    outs = {}
    for variant, dt in (("half", torch.float16), ("fp32", torch.float32)):
        hf = _hf_clip(tcfg, tsd, dt)
        with torch.no_grad():
            ctx = torch.cat([hf(input_ids=nids).last_hidden_state, hf(input_ids=ids).last_hidden_state]).half()
        ts, a_t, a_p = ddim_tables(3)
        cfgd = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(unet_cfg).items()}
        lref = denoise(RefUNet(cfgd, usd, None, variant=variant), lat, ctx, ts, a_t, a_p, 7.5)
        outs[variant] = (lref, postprocess(RefVAEDecoder(_vae_cfgdict(pipe.vae.config), vsd, None,
                                                         variant=variant).decode(lref)))
    _check_parity(lat_out, outs["half"][0], outs["fp32"][0], "tiny SD1.5 prompt -> latents (CLIP + 3 DDIM steps)")
    _check_parity(pt, outs["half"][1], outs["fp32"][1], "tiny SD1.5 prompt -> image")
    assert isinstance(pipe.vae, V.AutoencoderKL)


def test_tiny_sdxl_and_sd3_prompt_to_image():
    """SDXL: both encoders' penultimate states concatenated, pooled text_embeds of encoder 2, zero
    negative conditioning; SD3: CLIP-L | CLIP-G padded to the joint width + zero T5 tokens,
    16-channel VAE with shift.  Checked against transformers on the same weights."""
    from qdiff.clip import encode_sd3, encode_sdxl
    from qdiff.models import StableDiffusion3_5, StableDiffusionXL
    for cls, name in ((StableDiffusionXL, "synthetic:sdxl-tiny"), (StableDiffusion3_5, "synthetic:sd35-tiny")):
        model = cls.from_pretrained(name, device=DEV, seed=1)
        pipe = model.pipeline
        prompts = ["a red cube", "two dogs"]
        if cls is StableDiffusionXL:
            ctx, pooled = encode_sdxl(pipe, prompts)
            assert not ctx[:2].any() and not pooled[:2].any()     # force_zeros_for_empty_prompt
            e1 = _hf_outputs(_hf_clip(pipe.text_encoder.config, pipe.text_encoder.state_dict(), torch.float32),
                             pipe.tokenizer(prompts), pipe.text_encoder.config, -2, False)[0]
            h2, p2 = _hf_outputs(_hf_clip(pipe.text_encoder_2.config, pipe.text_encoder_2.state_dict(), torch.float32),
                                 pipe.tokenizer_2(prompts), pipe.text_encoder_2.config, -2, True)
            ref = torch.cat([e1, h2], -1)
            mx, _ = _rel_errs(ctx[2:], ref)
            pmx, _ = _rel_errs(pooled[2:], p2)
            assert mx < 5e-3 and pmx < 5e-3, (mx, pmx)
        else:
            jd = pipe.transformer.config.joint_attention_dim
            ctx, pooled = encode_sd3(pipe, prompts, joint_dim=jd)
            assert ctx.shape == (4, 154, jd) and pooled.shape == (4, pipe.transformer.config.pooled_projection_dim)
            assert not ctx[:, 77:].any()                               # zero T5 tokens
        hw = (pipe.unet if pipe.unet is not None else pipe.transformer).config.sample_size * 8
        img = model.generate(prompt=prompts, height=hw, width=hw, num_inference_steps=2, output_type="pt")
        assert img.shape == (2, 3, hw, hw) and torch.isfinite(img.float()).all()
        assert float(img.min()) >= 0 and float(img.max()) <= 1


def test_quantized_text_encoder_matches_oracle():
    """quantTextEncoder=True (W8A8 config): the CLIP linears are swapped like the UNet's; q/k/v
    carry the per-token output fake-quant (quantize/quantizer.py child-name rule).  Oracle:
    transformers' CLIP with the oracle's quantized weights and per-token output hooks."""
    from oracle import fake_quant_torch as FT
    from oracle.unet_ref import quantize_state_dict
    from qdiff.fake_quant import WxAxLinear
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:tiny", device=DEV, seed=6)
    pipe = model.pipeline
    te = pipe.text_encoder
    sd = {k: v.detach().cpu() for k, v in te.state_dict().items()}
    qc = dict(w_bit=8, a_bit=8, q_group_size=32, quantize_act=True)
    model.quantize(quant_config=dict(qc), quantUnet=False, quantTextEncoder=True)
    assert "text_encoder" in model.quantized_components
    assert isinstance(te.text_model.encoder.layers[0].self_attn.q_proj, WxAxLinear)
    qsd, flags = quantize_state_dict({k: v for k, v in sd.items() if "embedding" not in k}, qc)
    qsd.update({k: v for k, v in sd.items() if "embedding" in k})
    ids = pipe.tokenizer(["a quantized encoder", "second prompt here"])
    got, _ = te.encode(ids)
    refs = {}
    for variant, dt in (("half", torch.float16), ("fp32", torch.float32)):
        hf = _hf_clip(te.config, qsd, dt)
        for name, mod in hf.named_modules():
            f = flags.get("text_model." + name)
            if f and f.get("out_quant"):
                mod.register_forward_hook(lambda m, i, o, b=f["a_bit"]: FT.per_token(o.half(), b).to(o.dtype))
        with torch.no_grad():
            refs[variant] = hf(input_ids=ids).last_hidden_state
    _check_parity(got, refs["half"], refs["fp32"], "tiny CLIP W8A8-config quantized")
