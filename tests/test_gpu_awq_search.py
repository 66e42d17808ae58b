"""AWQ scale / clip search on the UNet (awq_search.py) against its CPU
restatement (oracle/awq_ref.py).  The searches pick an argmin over a grid, so parity is stated
on the loss landscape: every grid point's GPU loss equals the oracle's within 1 % (GEMM
accumulation order moves the fp16 outputs by ulps), and the GPU's choice is optimal for the
oracle up to that tolerance.  End to end: on a tiny SD1.5 the search runs over every
transformer block from a calibration run and the quantized UNet stays close to the fp16 one."""
import pytest
import torch

from oracle import awq_ref as AR

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _inputs(seed, t=2048, c=320, n_layers=3, n_out=320):
    g = torch.Generator().manual_seed(seed)
    # activation outlier channels (what AWQ protects): per-channel magnitudes spread over 30x
    mag = torch.exp(torch.randn(c, generator=g) * 1.2)
    x = (torch.randn(t, c, generator=g) * mag).half()
    ws = [(torch.randn(n_out, c, generator=g) / c ** 0.5).half() for _ in range(n_layers)]
    bs = [(torch.randn(n_out, generator=g) * 0.1).half() for _ in range(n_layers)]
    return x, ws, bs


@pytest.mark.parametrize("n_bits,group", [(4, 128), (4, 64), (8, 128)])
def test_scale_search_matches_oracle(n_bits, group):
    from torch import nn
    from qdiff.awq_search import search_scale
    x, ws, bs = _inputs(1 + n_bits + group)
    layers = []
    for w, b in zip(ws, bs):
        l = nn.Linear(w.shape[1], w.shape[0]).half().to(DEV)
        l.weight.data.copy_(w.to(DEV))
        l.bias.data.copy_(b.to(DEV))
        layers.append(l)
    s, r, hist = search_scale(x.to(DEV), layers, n_bits, group)
    ref, ref_scales = AR.scale_losses(x, ws, bs, n_bits, group)
    for k in ref:
        assert abs(hist[k] - ref[k]) <= 1e-2 * ref[k] + 1e-12, (k, hist[k], ref[k])
    best = min(ref.values())
    print(f"W{n_bits} g{group}: GPU ratio {r} loss {hist[r]:.4g} | oracle best {best:.4g} at "
          f"{min(ref, key=ref.get)} | ratio-0 {ref[0.0]:.4g}")
    assert ref[r] <= best * 1.01
    assert torch.allclose(s.cpu().float(), ref_scales[r].float(), rtol=2e-3, atol=0)
    assert best < ref[0.0]        # the activation-aware scales beat the weight-only ones here


@pytest.mark.parametrize("n_bits,group", [(4, 128), (3, 64)])
def test_clip_search_matches_oracle(n_bits, group):
    from qdiff.awq_search import N_GRID, search_clip
    x, ws, _ = _inputs(7 + group, n_layers=1, n_out=256)
    w = ws[0]
    best = search_clip(w.to(DEV), x.to(DEV), n_bits, group).cpu()
    co, ci = w.shape
    from qdiff.fake_quant import shrink_group
    g = shrink_group(ci, group)
    org = w.float().abs().view(co, ci // g, g).amax(-1)
    errs = torch.stack([AR.clip_errors(w, x, org * (1 - i / N_GRID), n_bits, group) for i in range(10)])
    emin = errs.min(0).values
    mine = AR.clip_errors(w, x, best, n_bits, group)
    shrunk = float((best < org.half().float() - 1e-6).float().mean())
    print(f"W{n_bits} g{group}: {shrunk:.0%} of (channel, group) clipped; err GPU-choice / oracle-min "
          f"max {float((mine / emin.clamp(min=1e-30)).max()):.4f}")
    ratio = mine / emin.clamp(min=1e-30)
    assert (mine <= emin * 1.03 + 1e-12).all() and float(ratio.mean()) <= 1.001
    assert shrunk > 0


def test_awq_search_tiny_unet_end_to_end():
    """quantize(quantType='awq', awq_search=True) on a tiny SD1.5: every block group searched and
    folded, clipping applied, the swap after it; the W4 UNet's output error against the fp16
    UNet stays within 1.25x of plain RTN's on the same input (random weights give AWQ little to
    gain; the bound catches a broken fold, which costs orders of magnitude)."""
    from qdiff import kernels as K
    from qdiff.models import StableDiffusion1_x

    def one_eval(model, x, ctx):
        unet = model.pipeline.unet
        kv = unet.prepare_context(ctx.to(DEV))
        temb = K.timestep_embedding(torch.tensor([601.0], device=DEV), None, x.shape[0], unet.config.block_out_channels[0])
        return K.nhwc_to_nchw(unet.fwd(K.nchw_to_nhwc(x.to(DEV), 8), temb, kv), 4).float().cpu()

    g = torch.Generator().manual_seed(5)
    ref_model = StableDiffusion1_x.from_pretrained("synthetic:tiny", device=DEV, seed=3)
    cfg = ref_model.pipeline.unet.config
    x = torch.randn(2, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    ctx = torch.randn(2, 77, cfg.cross_attention_dim, generator=g).half()
    y16 = one_eval(ref_model, x, ctx)
    qc = dict(w_bit=4, a_bit=16, q_group_size=32, quantize_act=False)
    errs = {}
    for search in (False, True):
        m = StableDiffusion1_x.from_pretrained("synthetic:tiny", device=DEV, seed=3)
        m.quantize(quant_config=dict(qc), quantUnet=True, awq_search=search,
                   calibration=dict(n_samples=4, batch_size=2, num_inference_steps=4))
        if search:
            rep = m.quantizer.search_report
            assert len(rep["scales"]) == 3 * len(m.get_smoothing_blocks()) and rep["clips"] > 0
            print("AWQ ratios:", {k: v["ratio"] for k, v in rep["scales"].items()})
        y = one_eval(m, x, ctx)
        errs[search] = float((y - y16).abs().mean() / y16.abs().mean())
    print(f"tiny SD1.5 W4 g32: rel. mean error vs fp16 - RTN {errs[False]:.4g}, AWQ search {errs[True]:.4g}")
    assert errs[True] <= 1.25 * errs[False]
