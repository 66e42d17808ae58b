"""CPU tests: the C-ABI library loads and exports every declared symbol; host-side logic
(config, traversal, module surface, scheduler tables, save/load files).  No kernel calls."""
import dataclasses
import json
import os
import re

import pytest
import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "qdiff.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|long|const char\*)\s+(qd_\w+)\(", src, re.M)))


def test_library_exports_all_declared_symbols():
    import ctypes
    from qdiff import _lib
    lib = _lib.load()
    decl = declared_symbols()
    assert len(decl) >= 25
    for name in decl:
        assert hasattr(lib, name), name
    # the ctypes table binds exactly the declared entry points
    assert sorted(_lib.exported_symbols()) == decl
    assert lib.qd_version() == 1


def test_bad_arguments_fail_before_launch():
    """Argument errors are reported with QD_ERR_ARG and a message, without touching a GPU."""
    import ctypes
    from qdiff import _lib
    with pytest.raises(RuntimeError, match="granularity"):
        _lib.call("qd_act_fakequant", ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 1, 8, 1, 1, 7, 0, 8,
                  ctypes.c_void_p(16), None)
    with pytest.raises(RuntimeError, match="n_bits"):
        _lib.call("qd_act_fakequant", ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 1, 8, 1, 1, 1, 0, 1,
                  ctypes.c_void_p(16), None)
    with pytest.raises(RuntimeError, match="K must be"):
        _lib.call("qd_linear_fwd", ctypes.c_void_p(16), 4, 12, 12, ctypes.c_void_p(16), 0, None, None, 0, None,
                  None, ctypes.c_void_p(16), 4, 4, 0, None, 0, None, 0, None)


def test_sd15_tree_matches_reference_counts():
    from qdiff.unet import SD15, UNet2DConditionModel
    u = UNet2DConditionModel(SD15)
    assert sum(isinstance(m, nn.Linear) for m in u.modules()) == 184
    assert sum(isinstance(m, nn.Conv2d) for m in u.modules()) == 98
    assert sum(p.numel() for p in u.parameters()) == 859_520_964          # SD1.5 UNet
    keys = u.state_dict().keys()
    for k in ("conv_in.weight", "time_embedding.linear_1.weight", "down_blocks.0.attentions.0.proj_in.weight",
              "down_blocks.0.attentions.0.transformer_blocks.0.attn2.to_k.weight",
              "down_blocks.0.attentions.0.transformer_blocks.0.ff.net.0.proj.weight",
              "down_blocks.0.downsamplers.0.conv.weight", "up_blocks.0.upsamplers.0.conv.weight",
              "up_blocks.3.resnets.2.conv_shortcut.weight", "mid_block.attentions.0.proj_out.bias",
              "conv_norm_out.weight", "conv_out.bias"):
        assert k in keys, k


def test_sdxl_tree_shape():
    from qdiff.unet import SDXL, UNet2DConditionModel
    u = UNet2DConditionModel(SDXL)
    n = sum(p.numel() for p in u.parameters())
    assert 2.55e9 < n < 2.6e9  # SDXL base UNet ~2.567 B
    assert sum(isinstance(m, nn.Linear) for m in u.modules()) == 743


def test_traversal_and_init_only_swap():
    """The reference traversal + init_only swap (base.py:658-692) on the SD1.5 tree, no kernels."""
    from qdiff.base import load_quantized_modules
    from qdiff.fake_quant import WxAxConv2d, WxAxLinear
    from qdiff.quantizer import MyTraversal
    from qdiff.unet import SD15, UNet2DConditionModel
    u = UNet2DConditionModel(SD15)
    found = []
    for name, child in u.named_children():
        t = MyTraversal()
        t.traverse(name, child, u)
        found += t.get_lin_conv()
    assert len(found) == 184 + 98
    sd_keys = set(u.state_dict().keys())
    load_quantized_modules(u, bitWidth=8, group_size=128, act_bits=8)
    assert sum(isinstance(m, WxAxLinear) for m in u.modules()) == 184
    convs = [m for m in u.modules() if isinstance(m, WxAxConv2d)]
    assert len(convs) == 98 and all(c.quantise_act for c in convs)  # base.py:688 forces it
    assert set(u.state_dict().keys()) == sd_keys  # reference-compatible buffer names
    assert "WxAxLinear(320, 320, bias=False, weight_quant=group, act_quant=per_token, output_quant=None)" in repr(u)


def test_module_errors():
    from qdiff.fake_quant import WxAxConv2d, WxAxLinear, shrink_group
    with pytest.raises(ValueError):
        WxAxLinear(8, 8, act_quant="per_channel")
    with pytest.raises(ValueError):
        WxAxConv2d(8, 8, 3, act_quant="bogus")
    with pytest.raises(ZeroDivisionError):
        shrink_group(36, 128)
    m = WxAxLinear(64, 64)
    with pytest.raises(RuntimeError, match="HIP tensor"):
        m(torch.zeros(2, 64, dtype=torch.float16))


def test_awq_config_roundtrip(tmp_path):
    from qdiff.config import AwqConfig
    c = AwqConfig.from_dict({"w_bit": 8, "a_bit": 8, "quantize_act": True, "version": "FAKE_ACT"})
    assert c.version == "fake_act" and c.q_group_size == 128 and c.weight_quant_conv_type == "per_channel"
    td = c.to_transformers_dict()
    assert td == {"quant_method": "awq", "zero_point": True, "group_size": 128, "bits": 8, "vbits": 4,
                  "act_bits": 8, "version": "fake_act", "modules_to_not_convert": None}
    back = AwqConfig(**AwqConfig.from_transformers_dict(AwqConfig, td))
    assert back.w_bit == 8 and back.a_bit == 8
    assert AwqConfig.from_pretrained(str(tmp_path), is_diffusion_model=True) == AwqConfig()
    with pytest.raises(TypeError):
        AwqConfig.from_dict({"bogus": 1})


def test_ddim_tables():
    from qdiff.scheduler import ddim_tables
    ts, a_t, a_p = ddim_tables(50)
    assert ts[0].item() == 981 and ts[-1].item() == 1 and len(ts) == 50
    assert torch.all(ts[:-1] - ts[1:] == 20)
    ts10, _, _ = ddim_tables(10)
    assert ts10.tolist() == [901, 801, 701, 601, 501, 401, 301, 201, 101, 1]
    assert a_p[-1].item() == pytest.approx(a_t.new_tensor(0).item() + a_p[-1].item())
    assert torch.all(a_p >= a_t)


def test_oracle_ddim_matches_formula():
    from oracle.unet_ref import ddim_step
    from qdiff.scheduler import ddim_tables
    ts, a_t, a_p = ddim_tables(50)
    g = torch.Generator().manual_seed(0)
    eps = torch.randn(4, 4, 8, 8, generator=g).half()
    lat = torch.randn(2, 4, 8, 8, generator=g).half()
    out = ddim_step(eps, 3, lat, a_t, a_p, 7.5).float()
    u, c = eps.float().chunk(2)
    e = u + 7.5 * (c - u)
    x0 = (lat.float() - (1 - a_t[3]).sqrt() * e) / a_t[3].sqrt()
    ref = a_p[3].sqrt() * x0 + (1 - a_p[3]).sqrt() * e
    assert (out - ref).abs().max() < 0.05 * ref.abs().max()


def test_synthetic_calibration_set():
    from qdiff.calib import synthetic_calibration_set
    s = synthetic_calibration_set(96, 8, 42)
    assert len(s) == 12 and s[0][1].shape == (8, 4, 64, 64) and s[0][1].dtype == torch.float16
    with pytest.raises(AssertionError):
        synthetic_calibration_set(10, 8)


def test_pipeline_files_roundtrip(tmp_path):
    """save_pretrained writes a diffusers-layout directory that load_pipeline reads back (CPU)."""
    from qdiff.pipeline_io import QDiffPipeline, load_pipeline
    from qdiff.unet import UNet2DConditionModel, tiny_config
    u = UNet2DConditionModel(tiny_config()).half().init_synthetic(3)
    QDiffPipeline(u).save_pretrained(str(tmp_path))
    assert json.load(open(tmp_path / "model_index.json"))["_class_name"] == "StableDiffusionPipeline"
    p = load_pipeline(str(tmp_path), device="cpu")
    for (k, a), (k2, b) in zip(u.state_dict().items(), p.unet.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    with pytest.raises(FileNotFoundError):
        load_pipeline(str(tmp_path / "nope"), device="cpu")


def test_euler_discrete_tables_match_oracle():
    from oracle.unet_ref import euler_tables
    from qdiff.scheduler import euler_discrete_tables
    for n in (4, 30, 50):
        ts, sig, dsc, init = euler_discrete_tables(n)
        ots, osig, oinit = euler_tables(n)
        assert torch.equal(ts, ots) and torch.equal(sig, osig) and init.item() == oinit.item()
        assert ts[0].item() == 1000 // n * (n - 1) + 1 and sig[-1].item() == 0.0 and len(sig) == n + 1
        assert torch.equal(dsc, (osig ** 2 + 1) ** 0.5)
    # SDXL base at 50 steps: sigma_max = sqrt((1 - acp[981]) / acp[981]) ~ 13.12
    _, sig, _, init = euler_discrete_tables(50)
    assert 13.0 < sig[0].item() < 13.3 and abs(init.item() - (sig[0].item() ** 2 + 1) ** 0.5) < 1e-4


def test_sdxl_tiny_tree_and_oracle_euler_runs():
    from oracle.unet_ref import RefUNet, denoise_euler, euler_tables
    from qdiff.unet import UNet2DConditionModel, tiny_sdxl_config
    cfg = tiny_sdxl_config()
    u = UNet2DConditionModel(cfg).half().init_synthetic(0)
    keys = set(u.state_dict())
    assert "add_embedding.linear_1.weight" in keys and "down_blocks.1.attentions.0.transformer_blocks.1.ff.net.2.bias" in keys
    assert u.state_dict()["add_embedding.linear_1.weight"].shape == (256, 64 + 6 * 32)
    cd = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}
    r = RefUNet(cd, dict(u.state_dict()))
    g = torch.Generator().manual_seed(0)
    add = r.add_embeds(torch.randn(2, 64, generator=g).half(), torch.tensor([[128.0, 128, 0, 0, 128, 128]] * 2))
    ts, sig, init = euler_tables(2)
    out = denoise_euler(r, torch.randn(1, 4, 16, 16, generator=g).half(), torch.randn(2, 77, 64, generator=g).half(),
                        add, ts, sig, init)
    assert out.shape == (1, 4, 16, 16) and torch.isfinite(out.float()).all()


def test_scheduler_config_roundtrip_and_pndm_tables(tmp_path):
    """A checkpoint's scheduler/scheduler_config.json selects the device loop's scheduler (the
    reference's generate() runs the pipeline's own scheduler, models/base.py:848): PNDM for SD1.5."""
    import json
    from oracle.unet_ref import PNDMRef, pndm_tables as oracle_tables
    from qdiff import pipeline_io as PIO
    from qdiff.scheduler import (DDIMConfig, EulerDiscreteConfig, PNDMConfig, config_from_diffusers,
                                 config_to_diffusers, pndm_tables)
    sd15 = {"_class_name": "PNDMScheduler", "beta_end": 0.012, "beta_schedule": "scaled_linear",
            "beta_start": 0.00085, "num_train_timesteps": 1000, "set_alpha_to_one": False, "skip_prk_steps": True,
            "steps_offset": 1, "trained_betas": None, "clip_sample": False}
    cfg = config_from_diffusers(sd15)
    assert isinstance(cfg, PNDMConfig) and cfg.skip_prk_steps
    for c in (cfg, DDIMConfig(), EulerDiscreteConfig()):
        assert config_from_diffusers(config_to_diffusers(c)) == c
    os_ = tmp_path / "scheduler"
    os_.mkdir()
    (os_ / "scheduler_config.json").write_text(json.dumps(sd15))
    assert isinstance(PIO.load_scheduler_config(str(tmp_path)), PNDMConfig)
    assert isinstance(PIO.load_scheduler_config(str(tmp_path), "ddim"), DDIMConfig)
    ts, a_t, a_p = pndm_tables(50)
    assert ts.tolist() == oracle_tables(50)[0].tolist() and len(ts) == 51
    r = PNDMRef()
    assert a_t[1].item() == r.ac[981].item() and a_p[1].item() == r.ac[961].item()   # counter-1 restart
    assert a_p[-1].item() == r.final.item()


def test_cpu_baseline_census_covers_the_unet():
    """The C1 CPU baseline times every op of a UNet evaluation: the census of the oracle's own
    forward finds SD1.5's 98 convs, 184 linears, 32 SDPA, 61 GroupNorms and 48 LayerNorms with the
    analytic FLOPs of SURVEY App. B (x CFG batch 2)."""
    import dataclasses
    from oracle import cpu_baseline as CB
    from qdiff.unet import SD15, UNet2DConditionModel
    with torch.device("meta"):
        net = UNet2DConditionModel(SD15)
    sd = {k: torch.empty(v.shape, dtype=torch.float16) for k, v in net.state_dict().items()}
    cd = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(SD15).items()}
    cen = CB.census(cd, sd)
    count, flop = {}, {}
    for (op, s), n in cen.items():
        count[op] = count.get(op, 0) + n
        flop[op] = flop.get(op, 0.0) + n * CB._flops(op, s)
    assert count == {"conv2d": 98, "linear": 184, "sdpa": 32, "group_norm": 61, "layer_norm": 48}
    assert abs(flop["conv2d"] / 2e9 - 443.9) < 1 and abs(flop["linear"] / 2e9 - 233.3) < 1
    assert abs(flop["sdpa"] / 2e9 - 126.1) < 1


def test_scheduler_configs_rejected_when_unsupported():
    """a DDIM / PNDM scheduler_config.json asking for trailing / linspace spacing,
    sample clipping or thresholding is refused rather than silently run as 'leading'."""
    import pytest
    from qdiff.scheduler import DDIMConfig, PNDMConfig, config_from_diffusers, config_to_diffusers
    base = {"beta_start": 0.00085, "beta_end": 0.012, "beta_schedule": "scaled_linear", "steps_offset": 1,
            "set_alpha_to_one": False}
    assert isinstance(config_from_diffusers({"_class_name": "DDIMScheduler", "clip_sample": False, **base}), DDIMConfig)
    assert isinstance(config_from_diffusers({"_class_name": "PNDMScheduler", "skip_prk_steps": True, **base}),
                      PNDMConfig)
    for bad in ({"_class_name": "DDIMScheduler", **base},                      # diffusers default clip_sample=True
                {"_class_name": "DDIMScheduler", "clip_sample": False, "timestep_spacing": "trailing", **base},
                {"_class_name": "PNDMScheduler", "timestep_spacing": "linspace", **base},
                # no timestep_spacing key: EulerDiscreteScheduler's diffusers default is "linspace"
                {"_class_name": "EulerDiscreteScheduler", **base},
                {"_class_name": "DDIMScheduler", "clip_sample": False, "thresholding": True, **base}):
        with pytest.raises(NotImplementedError):
            config_from_diffusers(bad)
    from qdiff.scheduler import EulerDiscreteConfig
    assert isinstance(config_from_diffusers({"_class_name": "EulerDiscreteScheduler", "timestep_spacing": "leading",
                                             **base}), EulerDiscreteConfig)
    for cfg in (DDIMConfig(), PNDMConfig(), EulerDiscreteConfig()):  # what save_pretrained writes reloads
        assert type(config_from_diffusers(config_to_diffusers(cfg))) is type(cfg)


def test_awq_clip_avoids_diffusers_qk_names():
    """the clip search skips the q / k projections under diffusers' names too
    (quantizer.py:788-791 avoids them by LLM substrings)."""
    from qdiff.awq_search import clip_avoided
    for n in ("attn1.to_q", "attn2.to_k", "attn.add_q_proj", "attn.add_k_proj", "self_attn.q_proj"):
        assert clip_avoided(n), n
    for n in ("attn1.to_v", "attn1.to_out.0", "ff.net.0.proj", "ff.net.2", "attn.add_v_proj"):
        assert not clip_avoided(n), n


def test_committed_gemm_table_loads():
    """The MI355X-tuned GEMM table (scripts/tune_table.py) is committed, well-formed and loaded at
    import, so every process runs the same kernel variant per shape."""
    import json
    import os
    from qdiff import kernels as K
    path = os.path.join(os.path.dirname(K.__file__), "gemm_table.json")
    d = json.load(open(path))
    assert d["device_arch"].startswith("gfx950") and len(d["entries"]) > 500
    kinds = {e[0][0] for e in d["entries"]}
    assert {"conv", "linear", "conv_i8", "linear_i8", "linear_fp8"} <= kinds
    if os.environ.get("QD_GEMM_TABLE", "").lower() != "none":
        assert len(K.gemm_choices()) >= len(d["entries"])
