"""BASELINE config C2 - the headline bench workload - at its own size (VERDICT r2 "top_next"):
SD1.5 W8A8 SmoothQuant, 512x512, 4 prompts per GPU (CFG batch 8), in both W8A8 modes.

  * fake-quant (the reference's arithmetic, bench.py's default line): the SmoothQuant fold and the
    quantized buffers equal the oracle's bit for bit; one UNet evaluation is within the
    self-calibrated bound of the committed half AND fp32 oracle outputs
    (tests/golden/config_golden.safetensors, case "c2"); and a teacher-forced pass over the FUSED
    launch sequence of that evaluation: every libqdiff launch unet.fwd makes (GEMM / conv with their
    bias / residual / GEGLU / amax epilogues, GroupNorm with the pending block-output finalize,
    LayerNorm with proj_in's pending fake-quant, attention, the fake-quant passes) is checked, at
    the shapes and kernel variants the bench runs, against oracle/fused_ref.py's restatement of
    the reference ops it fuses, fed the launch's own inputs;
  * int8-MFMA mode: every int8 layer bit-exact to oracle/int8_ref.py fed that
    layer's oracle input, and the whole evaluation within the self-calibrated bound of the int8
    oracle (half and fp32).

SmoothQuant statistics: the 600-eval calibration run is replaced by the fixed per-channel
activation absmax vectors of oracle/config_cases.sq_acts (stored in the fixture), fed to the
product's own SqQuantizer through its calibration hooks - quantizer_SQ.py:323-391, 395-431.
"""
import inspect
import json
import os
import time

import pytest
import torch

from oracle import config_cases as CC
from oracle import fused_ref as FR

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config_golden.safetensors")
QC = CC.CASES["c2"]["qc"]


def _golden():
    from safetensors import safe_open
    with safe_open(GOLDEN, "pt") as f:
        meta = json.loads(f.metadata()["c2"])
        acts = {k[len("c2.act."):]: f.get_tensor(k) for k in f.keys() if k.startswith("c2.act.")}
        return f.get_tensor("c2.half"), f.get_tensor("c2.fp32"), meta, acts


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
          f"oracle spread max {smx:.4g} mean {smean:.4g}", flush=True)
    tmx, tmean = 1.5 * smx + 2e-3, 1.5 * smean + 2e-3
    assert mx <= tmx and mean <= tmean, (mx, mean, tmx, tmean)
    assert mx32 <= tmx and mean32 <= tmean, (mx32, mean32, tmx, tmean)


def _sq_model(int8_mfma=False):
    """synthetic:sd15 -> SqQuantizer (quantType 'sq') with the fixture's activation statistics in
    the calibration hooks -> W8A8 swap.  Returns (model, unquantized CPU state dict)."""
    from qdiff.models import StableDiffusion1_x
    _, _, meta, gacts = _golden()
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=DEV, seed=0)
    unet = model.pipeline.unet
    sd = {k: v.detach().cpu() for k, v in unet.state_dict().items()}
    fp = CC.fingerprint(sd)
    assert abs(fp - meta["fingerprint"]) <= 1e-9 * max(1.0, abs(meta["fingerprint"])), (fp, meta["fingerprint"])
    acts = CC.sq_acts("c2", unet.config)
    blocks = model.get_smoothing_blocks()
    assert list(blocks) == CC.smoothing_blocks(unet.config) == list(acts)
    for p, (a1, a3) in acts.items():
        assert torch.equal(a1, gacts[p + ".norm1"]) and torch.equal(a3, gacts[p + ".norm3"]), p

    def fixed_statistics(**kw):  # stands in for run_sq_calibration: one "call" per hook
        for p, blk in blocks.items():
            a1, a3 = acts[p]
            for lin, a in ((blk.attn1.to_q, a1), (blk.attn1.to_k, a1), (blk.attn1.to_v, a1),
                           (blk.ff.net[0].proj, a3)):
                lin._qd_hook.sum.copy_(a.float().to(DEV))
                lin._qd_hook.count = 1

    model.run_sq_calibration = fixed_statistics
    model.quantize(quant_config=dict(QC), quantType="sq", quantUnet=True, int8_mfma=int8_mfma)
    return model, sd


def _inputs(unet):
    inp = CC.inputs("c2", unet.config)
    return inp["x"], CC.CASES["c2"]["t"], inp["ctx"]


def _eval(model, x, t, ctx):
    from qdiff import kernels as K
    unet = model.pipeline.unet
    kv = unet.prepare_context(ctx.to(DEV))
    xh = K.nchw_to_nhwc(x.to(DEV), 8)
    temb = K.timestep_embedding(torch.tensor([float(t)], device=DEV), None, x.shape[0],
                                unet.config.block_out_channels[0])
    return K.nhwc_to_nchw(unet.fwd(xh, temb, kv), 4).cpu()


@pytest.fixture(scope="module")
def c2():
    t0 = time.time()
    model, sd = _sq_model()
    print(f"[c2] model + SmoothQuant W8A8 {time.time() - t0:.1f}s", flush=True)
    return dict(model=model, sd=sd)


def test_c2_sq_fold_and_buffers_bit_exact(c2):
    """The SmoothQuant fold (LayerNorm / q,k,v / ff.net.0.proj) and every fake-quantized buffer
    equal the oracle's sq_fold + quantize_state_dict of the same weights, bit for bit."""
    from oracle.unet_ref import quantize_state_dict
    unet = c2["model"].pipeline.unet
    folded = CC.sq_fold(c2["sd"], CC.sq_acts("c2", unet.config), CC.CASES["c2"]["sq_alpha"])
    qsd, _ = quantize_state_dict(folded, dict(QC))
    got = unet.state_dict()
    assert set(got) == set(qsd)
    bad = [k for k, v in qsd.items() if not torch.equal(got[k].cpu().view(torch.int16), v.view(torch.int16))]
    nfold = sum(1 for k in folded if not torch.equal(folded[k], c2["sd"][k]))
    print(f"[c2] {len(qsd)} tensors compared, {nfold} changed by the fold, mismatching {len(bad)}")
    # per block: norm1 / norm3 weights + to_q / to_k / to_v / ff.net.0.proj weights (the synthetic
    # LayerNorm biases are 0, which the fold leaves 0)
    assert nfold == 16 * 6 and not bad, bad[:10]


@pytest.mark.timeout(600)
def test_c2_eval_matches_golden(c2):
    ref, ref32, _, _ = _golden()
    x, t, ctx = _inputs(c2["model"].pipeline.unet)
    got = _eval(c2["model"], x, t, ctx)
    again = _eval(c2["model"], x, t, ctx)
    assert got.shape == (8, 4, 64, 64) and torch.isfinite(got.float()).all()
    assert torch.equal(got, again)
    from bench import linear_families
    print(f"[c2] linear GEMM families: {linear_families()}", flush=True)
    _check_parity(got, ref, ref32, "C2 SD1.5 W8A8-SQ 512^2, 4 prompts (CFG 8) one eval")


@pytest.mark.timeout(900)
def test_c2_fused_launch_sequence_teacher_forced(c2):
    """Every libqdiff launch of one C2 evaluation (eager: the launch sequence the step graph
    captures), checked against oracle/fused_ref.py fed the launch's own inputs."""
    from qdiff import kernels as K
    model = c2["model"]
    x, t, ctx = _inputs(model.pipeline.unet)
    _eval(model, x, t, ctx)  # tune every GEMM shape first: the checked pass runs the chosen variants
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    stats, fails, counts = {}, [], {}
    orig = {name: getattr(K, name) for name in FR.LAUNCHES}

    def cpu(v):
        if isinstance(v, torch.Tensor):
            return v.detach().cpu().clone()
        if isinstance(v, tuple):
            return tuple(cpu(e) for e in v)
        return v

    def spy(name, fn):
        sig = inspect.signature(fn)

        def call(*a, **kw):
            bound = sig.bind(*a, **kw)
            bound.apply_defaults()
            torch.cuda.synchronize()
            args = {k: cpu(v) for k, v in bound.arguments.items() if k != "out"}
            ret = fn(*a, **kw)
            torch.cuda.synchronize()
            rets = list(ret) if isinstance(ret, tuple) else [ret]
            outs = FR.LAUNCHES[name](args, [cpu(r) for r in rets])
            got = {}
            i = 0
            for o in outs:
                if o.name == "amax" and name in ("linear", "conv2d_nhwc"):
                    got[o.name] = bound.arguments["amax"].detach().cpu()
                else:
                    got[o.name] = rets[i].detach().cpu()
                    i += 1
            idx = counts.get(name, 0)
            counts[name] = idx + 1
            for o in outs:
                ratio, beyond1, bad = FR.compare(got[o.name].reshape(o.ref.shape), o)
                key = f"{name}#{idx}.{o.name}"
                stats[key] = ratio
                if bad or beyond1 > 0.01:
                    fails.append((key, tuple(o.ref.shape), ratio, beyond1, bad))
            return ret
        return call

    for name, fn in orig.items():
        setattr(K, name, spy(name, fn))
    t0 = time.time()
    try:
        _eval(model, x, t, ctx)
    finally:
        for name, fn in orig.items():
            setattr(K, name, fn)
    top = sorted(stats.items(), key=lambda kv: -kv[1])[:8]
    print(f"[c2] fused launches checked in {time.time() - t0:.1f}s: {dict(sorted(counts.items()))}; "
          f"largest |err| / bound: " + ", ".join(f"{k} {v:.2f}" for k, v in top), flush=True)
    # every fused form the bench's step runs at this workload was exercised
    for name in ("linear", "linear_ln", "conv2d_nhwc", "groupnorm_fin", "groupnorm_nhwc", "layernorm", "layernorm_fq",
                 "attention"):
        assert counts.get(name, 0) > 0, (name, counts)
    assert counts["attention"] == 32, counts
    assert not fails, fails[:12]


# ------------------------------------------------------------------ int8-MFMA mode at C2
@pytest.fixture(scope="module")
def c2_int8():
    from oracle.unet_ref import RefUNet
    t0 = time.time()
    model, sd = _sq_model(int8_mfma=True)
    unet = model.pipeline.unet
    x, t, ctx = _inputs(unet)
    got = _eval(model, x, t, ctx)
    print(f"[c2 int8] model + gpu eval {time.time() - t0:.1f}s", flush=True)
    folded = CC.sq_fold(sd, CC.sq_acts("c2", unet.config), CC.CASES["c2"]["sq_alpha"])
    ref = RefUNet(CC.cfgdict(unet.config), folded, dict(QC), variant="fp32", int8=True)
    ref.record = rec = {}
    ref32 = ref.forward(x, t, ctx)
    ref.record = None
    ref.ops = torch.nn.functional  # the "half" variant of the same oracle (torch-CPU Half non-int8 ops)
    ref16 = ref.forward(x, t, ctx)
    print(f"[c2 int8] int8 oracles (fp32 + half) {time.time() - t0:.1f}s", flush=True)
    return dict(model=model, got=got, ref32=ref32, ref16=ref16, record=rec, i8=set(ref.i8))


@pytest.mark.timeout(900)
def test_c2_int8_eval_matches_int8_oracle(c2_int8):
    f = c2_int8
    assert f["got"].shape == (8, 4, 64, 64) and torch.isfinite(f["got"].float()).all()
    _check_parity(f["got"], f["ref16"], f["ref32"], "C2 int8-MFMA W8A8-SQ one eval vs int8 oracle")


@pytest.mark.timeout(900)
def test_c2_int8_teacher_forced_bit_exact(c2_int8):
    """Every int8 layer at CFG batch 8, fed the int8 oracle's input of that layer, reproduces its
    output bit for bit (the variants the tuner picks at M = 8 x H x W included)."""
    from qdiff import kernels as K
    from qdiff.unet import run_conv, run_linear
    f = c2_int8
    unet = f["model"].pipeline.unet
    n = {"conv": 0, "linear": 0}
    bad = []
    for name, tens in f["record"].items():
        if name not in f["i8"]:
            continue
        mod = unet.get_submodule(name)
        x, y = tens
        if hasattr(mod, "kernel_size"):
            n["conv"] += 1
            up = name.endswith("upsamplers.0.conv")
            xin = x[:, :, ::2, ::2].contiguous() if up else x
            got = K.nhwc_to_nchw(run_conv(mod, K.nchw_to_nhwc(xin.contiguous().to(DEV), mod.ci_pad), upsample=up)).cpu()
        else:
            if x.numel() // x.shape[-1] < 64:
                continue
            n["linear"] += 1
            got = run_linear(mod, x.reshape(-1, x.shape[-1]).contiguous().to(DEV)).view(*y.shape).cpu()
        if not torch.equal(got.view(torch.int16), y.view(torch.int16)):
            bad.append((name, (got.float() - y.float()).abs().max().item()))
    print(f"[c2 int8] layers checked: {n}, mismatching: {len(bad)}")
    assert n["conv"] > 90 and n["linear"] > 150, n
    assert not bad, bad[:10]
