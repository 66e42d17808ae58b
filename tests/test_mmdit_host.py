"""CPU tests of the SD3 / SD3.5 MMDiT host side: module tree and parameter counts of the
published configs (built on the meta device), state-dict names, quantizer traversal and the
output-quant naming rule, flow-match scheduler tables, the oracle's own consistency, and the
pipeline file round trip.  No kernel calls."""
import dataclasses
import json

import pytest
import torch
from torch import nn


def _meta(cfg):
    from qdiff.mmdit import SD3Transformer2DModel
    with torch.device("meta"):
        return SD3Transformer2DModel(cfg)


def test_sd35_large_and_sd3_medium_trees():
    from qdiff.mmdit import SD3_MEDIUM, SD35_LARGE
    m = _meta(SD35_LARGE)
    # 37 full blocks x 14 linears + the context_pre_only block's 11 + 7 embedding / output linears
    assert sum(isinstance(x, nn.Linear) for x in m.modules()) == 37 * 14 + 11 + 7
    assert sum(isinstance(x, nn.Conv2d) for x in m.modules()) == 1
    assert sum(p.numel() for p in m.parameters()) == 8_056_627_520          # SD3.5-Large, "8.1 B"
    assert sum(p.numel() for p in _meta(SD3_MEDIUM).parameters()) == 2_028_328_000   # SD3-Medium, "2 B"
    keys = set(m.state_dict().keys())
    for k in ("pos_embed.pos_embed", "pos_embed.proj.weight", "time_text_embed.timestep_embedder.linear_1.weight",
              "time_text_embed.text_embedder.linear_2.bias", "context_embedder.weight",
              "transformer_blocks.0.norm1.linear.weight", "transformer_blocks.0.norm1_context.linear.weight",
              "transformer_blocks.0.attn.add_q_proj.weight", "transformer_blocks.0.attn.norm_added_k.weight",
              "transformer_blocks.0.attn.to_add_out.bias", "transformer_blocks.0.ff_context.net.2.weight",
              "transformer_blocks.37.attn.to_out.0.weight", "norm_out.linear.weight", "proj_out.bias"):
        assert k in keys, k
    assert "transformer_blocks.37.attn.to_add_out.weight" not in keys
    assert "transformer_blocks.37.ff_context.net.0.proj.weight" not in keys
    assert m.state_dict()["transformer_blocks.37.norm1_context.linear.weight"].shape == (2 * 2432, 2432)


def test_traversal_swap_and_output_quant_names():
    """The reference traversal + init_only swap (base.py:658-692) on a tiny MMDiT: every Linear
    becomes WxAxLinear, and exactly the add_{q,k,v}_proj names get an output quant."""
    from qdiff.base import load_quantized_modules
    from qdiff.fake_quant import WxAxConv2d, WxAxLinear
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    m = SD3Transformer2DModel(tiny_mmdit_config(num_layers=3))
    n_lin = sum(isinstance(x, nn.Linear) for x in m.modules())
    keys = set(m.state_dict().keys())
    load_quantized_modules(m, bitWidth=4, group_size=128, act_bits=8)
    lin = {n: x for n, x in m.named_modules() if isinstance(x, WxAxLinear)}
    assert len(lin) == n_lin == 2 * 14 + 11 + 7
    assert sum(isinstance(x, WxAxConv2d) for x in m.modules()) == 1
    oq = sorted(n for n, x in lin.items() if x.output_quant_name != "None")
    assert oq == sorted(f"transformer_blocks.{i}.attn.add_{p}_proj" for i in range(3) for p in "qkv")
    assert set(m.state_dict().keys()) == keys


def test_flowmatch_tables_match_oracle_and_known_values():
    from oracle.mmdit_ref import flowmatch_tables as oracle_tables
    from qdiff.scheduler import FlowMatchConfig, flowmatch_tables
    for n in (4, 28, 50):
        ts, sig = flowmatch_tables(n)
        ots, osig = oracle_tables(n)
        assert torch.equal(ts, ots) and torch.equal(sig, osig)
        assert len(ts) == n and len(sig) == n + 1 and sig[-1].item() == 0.0 and ts[0].item() == 1000.0
        assert torch.all(sig[:-1] > sig[1:])
    ts, sig = flowmatch_tables(28)
    assert ts[1].item() == pytest.approx(987.3806, abs=1e-3)    # diffusers SD3 28-step schedule
    # shift 1.0: sigmas are the plain linspace
    _, s1 = flowmatch_tables(10, FlowMatchConfig(shift=1.0))
    assert torch.allclose(s1[:-1], torch.linspace(1.0, 0.001, 10), atol=1e-6)


def test_oracle_euler_step_formula():
    from oracle.mmdit_ref import euler_step, flowmatch_tables
    _, sig = flowmatch_tables(10)
    g = torch.Generator().manual_seed(0)
    mo = torch.randn(4, 16, 8, 8, generator=g).half()
    lat = torch.randn(2, 16, 8, 8, generator=g).half()
    out = euler_step(mo, 2, lat, sig, 7.0).float()
    u, c = mo.float().chunk(2)
    ref = lat.float() + (sig[3] - sig[2]) * (u + 7.0 * (c - u))
    assert (out - ref).abs().max() < 0.02 * ref.abs().max()


@pytest.mark.parametrize("dual", [(), (0, 1)])
def test_oracle_variants_agree_unquantized(dual):
    """Without activation quantization the oracle's fp16 and fp32 variants stay within a few ulp
    of each other on the tiny MMDiT (sanity of the restatement's op order); dual = MMDiT-X blocks."""
    from oracle.mmdit_ref import RefMMDiT
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    cfg = tiny_mmdit_config(num_layers=3, dual_attention_layers=dual) if dual else tiny_mmdit_config()
    t = SD3Transformer2DModel(cfg).half().init_synthetic(0)
    sd = dict(t.state_dict())
    cd = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 16, 16, 16, generator=g).half()
    enc = torch.randn(2, 40, 64, generator=g).half()
    pooled = torch.randn(2, 64, generator=g).half()
    a = RefMMDiT(cd, sd).forward(x, 1000.0, enc, pooled).float()
    b = RefMMDiT(cd, sd, variant="fp32").forward(x, 1000.0, enc, pooled).float()
    assert a.shape == (2, 16, 16, 16) and torch.isfinite(a).all()
    assert (a - b).abs().max() < 0.02 * a.abs().max()


def test_sd35_medium_tree():
    """SD3.5-Medium (MMDiT-X): blocks 0-12 carry SD35AdaLayerNormZeroX (9C adaLN) and an
    image-only attn2 (to_q/k/v/out + RMSNorm qk-norm).  2,243,171,520 parameters = SD3-Medium's
    2,028,328,000 + 13 x (4 attn2 linears + 3C extra adaLN rows) + the qk-norm weights."""
    from qdiff.base import load_quantized_modules
    from qdiff.fake_quant import WxAxLinear
    from qdiff.mmdit import SD35_MEDIUM, tiny_mmdit_config, SD3Transformer2DModel
    m = _meta(SD35_MEDIUM)
    assert sum(p.numel() for p in m.parameters()) == 2_243_171_520
    assert sum(isinstance(x, nn.Linear) for x in m.modules()) == 23 * 14 + 11 + 7 + 13 * 4
    sd = m.state_dict()
    assert sd["transformer_blocks.12.norm1.linear.weight"].shape == (9 * 1536, 1536)
    assert sd["transformer_blocks.13.norm1.linear.weight"].shape == (6 * 1536, 1536)
    assert "transformer_blocks.12.attn2.norm_k.weight" in sd and "transformer_blocks.13.attn2.to_q.weight" not in sd
    # reference naming rule: attn2.to_q / to_k / to_v do not contain "q_proj" -> no output quant
    t = SD3Transformer2DModel(tiny_mmdit_config(num_layers=3, dual_attention_layers=(0, 1)))
    load_quantized_modules(t, bitWidth=4, group_size=128, act_bits=8)
    oq = sorted(n for n, x in t.named_modules() if isinstance(x, WxAxLinear) and x.output_quant_name != "None")
    assert oq == sorted(f"transformer_blocks.{i}.attn.add_{p}_proj" for i in range(3) for p in "qkv")


def test_oracle_dual_block_with_silent_attn2_equals_plain_block():
    """Oracle self-consistency of the MMDiT-X restatement: with attn2.to_out zeroed the attn2
    residual adds exact zeros, so the dual model equals the plain model holding the first 6C
    adaLN rows, bit for bit."""
    from oracle.mmdit_ref import RefMMDiT
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    cd_ = tiny_mmdit_config(num_layers=3, dual_attention_layers=(0, 1))
    cp_ = tiny_mmdit_config(num_layers=3)
    t = SD3Transformer2DModel(cd_).half().init_synthetic(4)
    sd = dict(t.state_dict())
    c = cd_.inner_dim
    for i in (0, 1):
        sd[f"transformer_blocks.{i}.attn2.to_out.0.weight"] = torch.zeros_like(sd[f"transformer_blocks.{i}.attn2.to_out.0.weight"])
    plain = {k: v for k, v in sd.items() if ".attn2." not in k}
    for i in (0, 1):
        for w in ("weight", "bias"):
            plain[f"transformer_blocks.{i}.norm1.linear.{w}"] = sd[f"transformer_blocks.{i}.norm1.linear.{w}"][:6 * c]
    assert set(plain) == set(SD3Transformer2DModel(cp_).state_dict())
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 16, 16, 16, generator=g).half()
    enc = torch.randn(2, 24, 64, generator=g).half()
    pooled = torch.randn(2, 64, generator=g).half()
    asd = lambda cfg: {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}
    a = RefMMDiT(asd(cd_), sd).forward(x, 700.0, enc, pooled)
    b = RefMMDiT(asd(cp_), plain).forward(x, 700.0, enc, pooled)
    assert torch.equal(a, b)
    # and the attn2 branch is live when its weights are not zero
    sd2 = dict(t.state_dict())
    assert not torch.equal(RefMMDiT(asd(cd_), sd2).forward(x, 700.0, enc, pooled), a)


def test_mmdit_pipeline_files_roundtrip(tmp_path):
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    from qdiff.pipeline_io import QDiffPipeline, load_config, load_pipeline
    t = SD3Transformer2DModel(tiny_mmdit_config()).half().init_synthetic(3)
    p = QDiffPipeline(transformer=t, class_name="StableDiffusion3Pipeline")
    assert set(p.components) >= {"transformer", "text_encoder", "vae", "scheduler"}
    p.save_pretrained(str(tmp_path))
    idx = json.load(open(tmp_path / "model_index.json"))
    assert idx["_class_name"] == "StableDiffusion3Pipeline" and "transformer" in idx
    q = load_pipeline(str(tmp_path), device="cpu")
    assert q.unet is None
    for (k, a), (k2, b) in zip(t.state_dict().items(), q.transformer.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    assert load_config("synthetic:sd35")["_class_name"] == "StableDiffusion3Pipeline"
    with pytest.raises(ValueError):
        QDiffPipeline()


def test_sd35_adapter_surface():
    from qdiff.mmdit import SD3Transformer2DModel, tiny_mmdit_config
    from qdiff.models import CLASS_MAP, StableDiffusion3_5
    from qdiff.pipeline_io import QDiffPipeline
    t = SD3Transformer2DModel(tiny_mmdit_config()).half()
    a = StableDiffusion3_5(QDiffPipeline(transformer=t, class_name="StableDiffusion3Pipeline"),
                           "StableDiffusion3Pipeline", False, {}, None)
    assert CLASS_MAP["StableDiffusion3Pipeline"] is StableDiffusion3_5
    assert a.get_components()["transformer"] == ["transformer"]
    assert [n for n, _ in a.get_model_layers_transformers()[0]][:3] == ["pos_embed", "time_text_embed",
                                                                      "context_embedder"]
    with pytest.raises(Exception, match="NO UNET"):
        a.get_model_layers_unet()
    with pytest.raises(Exception, match="no UNET"):
        a.checkQuantStatus(quantUnet=True)
    with pytest.raises(Exception, match="refiner"):
        StableDiffusion3_5(None, "x", False, {}, None, refiner_path="r")
