"""bench.py - images/s of the SD1.5 W8A8 (SmoothQuant fake-quant) 512x512 batch-4 50-step
denoising loop on MI355X (BASELINE.json metric / configs[1]), 1..N GPUs of one node.

One "step" = one generate() over the per-GPU batch: RCCL broadcast of the text embeddings
from rank 0, 50 graph-replayed denoising steps (UNet on the CFG batch 2B, CFG combine, DDIM),
gather of the final latents.  Weak scaling: every rank denoises B=4 prompts per step.

Also reported (rank 0):
  roofline      the dominant kernel (the largest conv implicit GEMM of the UNet) timed live
                with HIP events on the stream it runs on; ALGORITHMIC flops / duration vs the
                fp16 dense MFMA peak (the path computes fake-quant operands in fp16)
  path_roofline whole-loop FLOP rate (803.3 GFLOP per UNet eval per sample)
  cpu_baseline  BASELINE.md §2: the reference's CPU path (config C1) restated by the oracle
                (torch-CPU fp16 ops) timed on this box's host cores: every distinct op shape of a
                UNet evaluation on a bounded slice, warm-up + median of 3 (see cpu_baseline())
  int8_blended_roofline  images/s against the int8-MFMA-blended bound of north_star's target
Secondary lines (same JSON contract): --model sdxl (SURVEY config C4: SDXL W8A8 1024^2, 2
prompts per GPU, 50 EulerDiscrete steps) and --model sd35 (config C5: SD3.5-Large W4A16 g128
1024^2, 1 prompt per GPU, flow-match Euler).
Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model sd15|sdxl|sd35]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

UNET_GFLOP_PER_SAMPLE = 803.3   # SURVEY.md Appendix B (analytic, SD1.5 512^2)
PEAK_F16_TFLOPS = 2500.0        # MI355X_MICROARCH.md: dense BF16/FP16 MFMA
PEAK_I8_TOPS = 5000.0           # MI355X_MICROARCH.md: I8 MFMA = 2x the BF16 rate per clock (dense)
# int8-eligible (quantized GEMM) and fp16 (attention) FLOP per SD1.5 512^2 image
SD15_I8_FLOP_PER_IMAGE, SD15_F16_FLOP_PER_IMAGE = 67.72e12, 12.61e12
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=4, help="prompts per GPU")
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--denoise-steps", type=int, default=50)
    ap.add_argument("--mode", default=None, choices=["w8a8-sq", "w8a8", "w4a16", "fp16", "w8a8-sq-int8", "w8a8-int8",
                                                     "w4a8-fp8"],
                    help="default: w8a8-sq (sd15), w4a16 (sd35, SURVEY config C5)")
    ap.add_argument("--model", default="sd15", choices=["sd15", "sdxl", "sd35"],
                    help="secondary lines: sdxl = SDXL W8A8 1024^2, 2 prompts per GPU (config C4); "
                         "sd35 = SD3.5-Large W4A16 1024^2, 1 prompt per GPU (config C5)")
    # SmoothQuant calibration: the reference's defaults (quantizer_SQ.py:331-339: 96 samples in
    # batches of 8, 50 denoising steps each = 600 UNet evaluations at CFG batch 16, eager, hooked)
    ap.add_argument("--calib-steps", type=int, default=50)
    ap.add_argument("--calib-samples", type=int, default=96)
    ap.add_argument("--calib-batch", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the text encoder + VAE end-to-end timing")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: every usable core (sched_getaffinity, capped by the cgroup CPU quota)")
    ap.add_argument("--epi-lds", action="store_true",
                    help="measurement: every GEMM epilogue through the LDS C tile (qd_gemm_epi_lds, A/B runs)")
    ap.add_argument("--gn-geom", default=None,
                    help="measurement: GroupNorm statistics / apply rows per thread 'S,A' (qd_gn_geom_force, A/B runs)")
    ap.add_argument("--no-int8-mode", action="store_true",
                    help="skip the int8-MFMA mode object of the default SD1.5 W8A8 line")
    a = ap.parse_args()
    if a.mode is None:
        a.mode = {"sd35": "w4a16", "sdxl": "w8a8"}.get(a.model, "w8a8-sq")
    if a.model == "sdxl":
        if a.res == 512:
            a.res = 1024
        if a.batch == 4:
            a.batch = 2
    if a.model == "sd35":
        if a.mode == "w8a8-sq":
            ap.error("SmoothQuant has no SD3.5 block mapping in the reference")
        if a.res == 512:
            a.res = 1024
        if a.batch == 4:
            a.batch = 1
    return a


QCFG = {
    "w8a8-sq": dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True),
    "w8a8": dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True),
    # the int8-MFMA W8A8 mode: same config, int8 codes on v_mfma_i32_16x16x64_i8
    "w8a8-sq-int8": dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True),
    "w8a8-int8": dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True),
    "w4a16": dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
    # SD3.5 (config C5's "fp8 activations on CDNA4"): W4 g128 codes as e4m3,
    # per-token e4m3 activations on v_mfma_scale_f32_16x16x128_f8f6f4
    "w4a8-fp8": dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
}
PEAK_F8_TFLOPS = 5000.0         # MI355X_MICROARCH.md: block-scaled fp8 MFMA = 2x the BF16 rate (dense)


def mmdit_gflop_per_sample(cfg, s, sc):
    """Analytic GFLOP of one SD3 transformer evaluation for one sample: token GEMMs (12 C^2 MACs
    per token per stream per block: q, k, v, out + 4C FF; the last block's context stream only
    its add_q/k/v 3 C^2) + joint attention (4 (S+Sc)^2 C) + patch embed / proj_out."""
    c, n = cfg.inner_dim, cfg.num_layers
    p2c = cfg.patch_size ** 2 * cfg.in_channels
    macs = n * 12 * c * c * s + (n - 1) * 12 * c * c * sc + 3 * c * c * sc + 2 * s * c * p2c
    return (2 * macs + n * 4 * (s + sc) ** 2 * c) / 1e9


def build_model(args, dev):
    if args.model == "sdxl":
        from qdiff.models import StableDiffusionXL
        model = StableDiffusionXL.from_pretrained("synthetic:sdxl", device=dev, seed=0)
        if args.mode == "w8a8-sq":
            model.quantize(quant_config=dict(QCFG[args.mode]), quantType="sq", quantUnet=True,
                           calibration=dict(n_samples=args.calib_samples, batch_size=args.calib_batch,
                                            num_inference_steps=args.calib_steps, height=args.res, width=args.res))
        elif args.mode != "fp16":
            model.quantize(quant_config=dict(QCFG[args.mode]), quantUnet=True)
        return model
    if args.model == "sd35":
        from qdiff.models import StableDiffusion3_5
        model = StableDiffusion3_5.from_pretrained("synthetic:sd35", device=dev, seed=0)
        if args.mode != "fp16":
            model.quantize(quant_config=dict(QCFG[args.mode]), quantTransformer=True, fp8_act=args.mode == "w4a8-fp8")
        return model
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    if args.mode != "fp16":
        qc = dict(QCFG[args.mode])
        i8 = args.mode.endswith("-int8")
        if args.mode.startswith("w8a8-sq"):
            model.quantize(quant_config=qc, quantType="sq", quantUnet=True, int8_mfma=i8,
                           calibration=dict(n_samples=args.calib_samples, batch_size=args.calib_batch,
                                            num_inference_steps=args.calib_steps))
        else:
            model.quantize(quant_config=qc, quantUnet=True, int8_mfma=i8)
    return model


ROOF_FLUSH_MB = 0  # a cache-evicting write between the int8 roofline launches (MB; 0 = none, the default)


def dominant_kernel_roofline(dev, iters=20, n=8, h=64, w=64, c=320, int8=False):
    """Time the largest conv implicit GEMM of the UNet (SD1.5 at CFG batch 8: down/up block 0
    conv 320->320 3x3 @ 64x64, M = 32768, N = 320, K = 2880; SDXL at CFG batch 4: the same conv
    at 128x128, M = 65536) with HIP events on its stream, in the form the captured step launches it
    (VERDICT r5 #2): the fake-quant conv with bias + the output fake-quant's per-(n, c) amax epilogue
    into a pre-zeroed pooled buffer (AMAX_ZEROED: no zero-fill launch, as the arena step); the int8-MFMA
    mode's resnet conv1 (qd_conv2d_i8 on per-sample codes) with bias, the time-embedding add (CADD)
    and the consumer GroupNorm's slot statistics (GNSTATS) - against the int8 MFMA peak."""
    import torch
    from qdiff import kernels as K
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(n, h, w, c, generator=g).half().to(dev)
    wt = (torch.randn(c, 3, 3, c, generator=g) / 54).half().to(dev)
    b = torch.zeros(c, dtype=torch.float16, device=dev)
    amax = torch.zeros(n * c, dtype=torch.float32, device=dev)
    # the input rotates over NROT copies (> the XCDs' aggregate 32 MB of L2): in the step each conv
    # reads an activation another kernel just wrote, not one its own previous launch left in L2
    NROT = 4
    if int8:
        xq, sa = K.quant_samples_i8(x)
        xqs = [xq] + [xq.clone() for _ in range(NROT - 1)]
        wq, sw16, _ = K.weight_quant(wt.view(c, -1).contiguous(), 9 * c, 8, want_dq=False)
        wq, sw = wq.view(c, 3, 3, c), sw16.float().view(-1).contiguous()
        temb = (torch.randn(n, c, generator=g) * 0.1).half().to(dev)
        run = lambda i: K.conv2d_i8(xqs[i % NROT], sa, wq, sw, c, 1, 1, bias=b, chan_add=temb, gn_stats=True)
    else:
        xs = [x] + [x.clone() for _ in range(NROT - 1)]
        run = lambda i: K.conv2d_nhwc(xs[i % NROT], wt, c, 1, 1, bias=b, amax=amax, amax_zeroed=True)
    for i in range(NROT):
        run(i)
    st = torch.cuda.current_stream()
    # Timed so that avg_us agrees with the step sequence's durations of the same launches
    # (scripts/roof_check.py, profiles/r06zb_roofline_forms.log): the int8 conv one launch per event
    # pair right after a copy writes its input (as the GroupNorm apply does in the step: 39.2 us vs
    # 38.4-40.2 in prof_r06z_int8; back to back on warm inputs it read 36.5); the fp16 conv back to
    # back over the rotated inputs (59.3 us vs 55.1-57.8; after a producer copy it read 62.7).
    if int8:
        flush = torch.empty(max(ROOF_FLUSH_MB, 1) << 19, dtype=torch.float16, device=dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for i in range(iters):
            if ROOF_FLUSH_MB:
                flush.zero_()
            xqs[i % NROT].copy_(xq)
            ev[i][0].record(st)
            run(i)
            ev[i][1].record(st)
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in ev) / iters
    else:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(iters):
            run(i)
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * (n * h * w) * c * (9 * c)
    tflops = flops / (ms * 1e-3) / 1e12
    peak = PEAK_I8_TOPS if int8 else PEAK_F16_TFLOPS
    choice = _conv_choice((n, h, w, c), "conv_i8" if int8 else "conv")
    tr = pmc_traffic(choice["variant"] if choice else None, int8) if (n, h, w, c) == (8, 64, 64, 320) else None
    return {"bound": "mfma", "achieved": round(tflops, 1), "peak": peak, "unit": "TOP/s" if int8 else "TFLOP/s",
            "frac": round(tflops / peak, 4), "traffic": (tr or {}).get("hbm_bytes_per_launch"),
            "traffic_unit": "bytes per launch (rocprofv3 PMC)", "traffic_detail": tr,
            "kernel": f"conv3x3 {c}->{c} @{h}x{w} b{n} (M={n * h * w},N={c},K={9 * c}) implicit GEMM"
                      + (" int8 x int8 -> int32 (v_mfma_i32_16x16x64_i8), bias + temb add + GroupNorm slot "
                         "statistics epilogue (the step's resnet conv1)" if int8 else
                         ", bias + output-fake-quant amax epilogue (the step's form)"),
            "kernel_choice": choice,
            "avg_us": round(ms * 1e3, 2)}


def _conv_choice(shape=(8, 64, 64, 320), kind="conv"):
    """GEMM family chosen for the dominant conv ((weight op, qd_gemm_force id); >= 100 = LDS-DMA)."""
    from qdiff import kernels as K
    n, h, w, c = shape
    for key, ch in K.gemm_choices().items():
        if kind == "conv_i8":
            # the step's conv1 form: bias | CADD | GNSTATS (kernels.conv2d_i8 key, last field = epi)
            if key[:8] == ("conv_i8", n, h, w, c, c, 3, 3) and key[-1] == (1 | 128 | 256):
                if not ch:
                    return None
                v = ch % 1000  # (+ 1000 * s: an explicit split-K count)
                fam = ("k_conv_halo_i8" if 140 <= v <= 149 else "k_gemm_pp<I8>" if 130 <= v <= 134 else
                       "k_gemm_dma<I8>")
                return {"variant": ch, "family": fam}
            continue
        if key[:8] == ("conv", n, h, w, c, c, 3, 3) and key[-1] == (1 | 4):  # bias | AMAX
            fam = ("k_gemm_pp" if ch and ch[1] >= 300 else "k_conv_halo" if ch and ch[1] >= 200 else
                   "k_gemm_dma" if ch and ch[1] >= 100 else "k_gemm")
            return {"variant": ch[1], "family": fam} if ch else None
    return None


def end_to_end(model, lat_nchw, prompts, step_s, reps=3):
    """Prompt -> image around the timed denoising loop (rank 0, same per-GPU batch): the CLIP
    text encoder on the prompts + "" negatives (the pipeline's encode_prompt) and the VAE decode
    of the loop's latents to uint8 images (output_type "pil" minus the PIL wrapping), each warmed
    up, then the median of `reps` timed runs; images/s = B / (loop step + encode + decode)."""
    import statistics
    import torch
    from qdiff import kernels as K
    vae = model.pipeline.vae
    lat = K.nchw_to_nhwc(lat_nchw.contiguous(), 8)

    def enc():
        return model._text_context(prompts, None, None, None)

    def dec():
        n, h, w, _ = lat.shape
        for i in range(0, n, vae.samples_per_chunk(h, w)):
            K.vae_postprocess(vae.decode_nhwc(lat[i:i + vae.samples_per_chunk(h, w)].contiguous()), 3,
                              want_nchw=False, want_u8=True)

    out = {}
    for name, fn in (("text_encode", enc), ("vae_decode", dec)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_ms"] = round(statistics.median(ts) * 1e3, 2)
    tot = step_s + (out["text_encode_ms"] + out["vae_decode_ms"]) / 1e3
    out["images_per_s"] = round(len(prompts) / tot, 4)
    out["note"] = (f"{len(prompts)} prompts: CLIP ViT-L/14 (12 layers, 77 tokens, + negatives) and the SD VAE decoder "
                   f"({lat.shape[1] * 8}^2 uint8 images), HIP path, synthetic weights; loop step {step_s * 1e3:.1f} ms")
    return out


def linear_families():
    """GEMM family the tuner chose for each linear shape of the loop, counted per operand:
    packed int4 / int8 codes dequantized in the register-tile staging (k_gemm) or the fp16
    dequantized copy through the LDS-DMA / ping-pong families; int8-MFMA linears separately."""
    from qdiff import kernels as K
    fam = {}
    for key, ch in K.gemm_choices(used_only=True).items():
        if ch is None:
            continue
        if key[0] == "linear_i8":
            name = "int8 codes -> k_gemm_dma<I8>"
        elif key[0] == "linear":
            fmt, v = key[-1][ch[0]], ch[1]
            kind = "k_gemm_pp" if v >= 300 else "k_gemm_dma" if v >= 100 else "k_gemm register tile"
            name = f"{key[-1][0]} weights: {fmt} operand -> {kind}"
        else:
            continue
        fam[name] = fam.get(name, 0) + 1
    return fam


def weight_footprint(model):
    """HBM bytes of the denoiser's linear weights per operand form (MB): the packed-int4 codes +
    group scales ([N][K/g] and the [K/g][N] copy the LDS-DMA stages read) vs the module's fp16
    dequantized buffer (the reference's `weight`, which the tuner may also stream), and which
    operand the linears' chosen kernels actually read; conv weights are fp16 [Co][kh][kw][Ci]."""
    from qdiff import kernels as K
    from qdiff.fake_quant import WxAxLinear
    codes = f16 = 0
    net = getattr(model.pipeline, "unet", None) or model.pipeline.transformer
    for m in net.modules():
        if isinstance(m, WxAxLinear) and m.qcodes is not None and m.qfmt == "i4":
            codes += m.qcodes.numel() + 2 * m.qscales.numel() * 2
            f16 += m.weight.numel() * 2
    ran = {"codes": 0, "f16 buffer": 0}
    for key, ch in K.gemm_choices(used_only=True).items():
        if key[0] == "linear" and key[-1][0] == "i4" and ch is not None:
            ran["codes" if key[-1][ch[0]] == "i4" else "f16 buffer"] += 1
    return {"int4_codes_and_scales_MB": round(codes / 2**20, 1), "fp16_buffer_MB": round(f16 / 2**20, 1),
            "linear_shapes_by_operand": ran,
            "operand_policy": "int4 codes only (QD_W4_OPERAND=codes)" if K.W4_CODES_ONLY else
            "tuned per shape: int4 codes vs the fp16 dequantized buffer (default)"}


def pmc_traffic(variant=None, int8=False):
    """HBM bytes per launch of the dominant kernel from the newest committed rocprofv3 --pmc
    measurement (profiles/*pmc_dominant.json: FETCH_SIZE x2 + WRITE_SIZE, separate passes over
    scripts/roof_kernel.py - the same kernel and shape as dominant_kernel_roofline(), per GEMM
    variant when the file holds several)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_dominant.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    if "by_variant" in d:
        rec = d["by_variant"].get(f"i8:{variant}" if int8 else str(variant))
        if rec is None:
            return None
        alg = d["algorithmic_bytes_per_launch_i8" if int8 else "algorithmic_bytes_per_launch"]
        return {"hbm_bytes_per_launch": rec["hbm_bytes_per_launch"], "kernel": rec["kernel_name"][:80],
                "read_bytes_per_launch": rec.get("read_bytes_per_launch"),
                "write_bytes_per_launch": rec.get("write_bytes_per_launch"),
                "algorithmic_bytes_per_launch": alg, "source": os.path.relpath(files[-1], ROOT)}
    if int8:
        return None
    return {"hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
            "algorithmic_bytes_per_launch": d["algorithmic_bytes_per_launch"],
            "source": os.path.relpath(files[-1], ROOT)}


def usable_cores():
    """(cores, note): the host cores this process may run on - the sched_getaffinity set, capped by
    the cgroup CPU quota when one is set (a GPU box shares its host: affinity lists every core of
    the machine while the quota grants this job a slice; threads beyond the quota only time-slice,
    and torch's CPU ops then run several times slower than on the quota's cores)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            quota = None
    env = os.environ.get("OMP_NUM_THREADS")
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    note = f"sched_getaffinity {aff} cores, cgroup CPU quota {quota if quota is not None else 'none'}"
    if quota is None and env and env.isdigit() and 0 < int(env) < aff:
        # no quota visible: the box's stated per-job CPU share (OMP_NUM_THREADS) bounds the threads
        cores = int(env)
        note += f", OMP_NUM_THREADS {env} (the job's CPU share)"
    return cores, note


def cpu_baseline(threads):
    """the reference's CPU fake-quant path on config C1 (SD1.5 W8 RTN, 1 prompt,
    512x512, 10 DDIM steps with CFG = 10 UNet evaluations at batch 2) restated by the oracle
    (torch-CPU fp16 ops, bit-exact per op to the reference's goldens), timed on this host's cores:
    every distinct op shape of one UNet evaluation (census of the oracle's own forward) on a
    bounded slice, 1 warm-up + median of 3, scaled by FLOPs and summed with multiplicities
    (oracle/cpu_baseline.py; a whole C1 run takes hours where torch's Half conv is scalar)."""
    import dataclasses
    import torch
    from oracle import cpu_baseline as CB
    from qdiff.unet import SD15, UNet2DConditionModel
    with torch.device("meta"):
        net = UNet2DConditionModel(SD15)
    shapes = {k: torch.empty(v.shape, dtype=torch.float16) for k, v in net.state_dict().items()}
    cd = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(SD15).items()}
    note = None
    usable, unote = usable_cores()
    if threads is None:
        threads, note = usable, unote
    elif threads > usable:  # (an explicit count above the affinity / quota oversubscribes: ADVICE r5)
        note = f"--cpu-threads {threads} capped to the {usable} usable cores ({unote})"
        threads = usable
    r = CB.c1_baseline(cd, shapes, threads=threads)
    pc = r["per_class"]
    return {"value": round(1.0 / r["seconds_per_image"], 8), "unit": "images/s", "cores": r["threads"],
            "cores_note": note or "--cpu-threads",
            "kind": "port", "cpu": r["cpu"], "config": "C1: SD1.5 W8 RTN fake-quant (A16), 1 prompt 512x512, "
                                                       "10 DDIM steps + CFG (10 UNet evals at batch 2)",
            "sample": (f"{r['distinct_shapes']} distinct op shapes / {r['ops_per_eval']} ops per UNet eval, each on a "
                       f"bounded slice (1 warm-up + median of 3, scaled by FLOPs): conv2d "
                       f"{pc['conv2d']['gflops']} GFLOP/s, linear {pc['linear']['gflops']} GFLOP/s, SDPA "
                       f"{pc['sdpa']['gflops']} GFLOP/s; {r['seconds_per_unet_eval']:.1f} s per eval; sampling wall "
                       f"{r['wall_s']:.1f} s; elementwise ops untimed (upper bound on CPU speed)"),
            "per_class": pc, "seconds_per_image": round(r["seconds_per_image"], 1)}


def launch_ranks(args):
    """`bench.py --gpus N` run directly (not under torchrun): this parent never touches the GPU;
    it starts N ranks (one process per GPU) through torch.distributed.run on 127.0.0.1 and exits
    with their status (non-zero if any rank failed)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist
    import qdiff_boot  # noqa: F401
    from qdiff import dist as qdist
    from qdiff.pipeline import synthetic_text_embeddings

    rank, world, local = qdist.init_from_env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: run `python bench.py --gpus N` "
                         "(it launches the N ranks itself) or torchrun with --nproc-per-node N")
    n_gpus = world
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    def log(msg):
        if rank == 0:
            print(f"[bench +{time.time() - T0:.0f}s] {msg}", file=sys.stderr, flush=True)

    T0 = time.time()
    if args.epi_lds:
        from qdiff import _lib
        _lib.call("qd_gemm_epi_lds", 1)
    if args.gn_geom:
        from qdiff import _lib
        _lib.call("qd_gn_geom_force", *[int(v) for v in args.gn_geom.split(",")])
    model = build_model(args, dev)
    log(f"model built + quantized ({args.model} {args.mode})")
    if args.model == "sd35":
        return main_sd35(args, model, rank, world, dev, log)
    if args.model == "sdxl":
        return main_sdxl(args, model, rank, world, dev, log)
    B = args.batch
    hw = args.res // 8
    loop = model.get_loop(B, args.res, args.res, args.denoise_steps, 7.5, use_graph=True)
    # full CFG context for all ranks' prompts, created on rank 0 and broadcast each step
    full_ctx = torch.empty(2 * B * world, 77, 768, dtype=torch.float16, device=dev)
    prompts = [f"a photograph of synthetic scene {i}" for i in range(B * world)]
    if rank == 0:
        full_ctx.copy_(torch.cat([synthetic_text_embeddings([""] * (B * world), device=dev),
                                  synthetic_text_embeddings(prompts, device=dev)]))
    g = torch.Generator().manual_seed(42 + rank)
    lat = torch.randn(B, 4, hw, hw, generator=g).half().to(dev)

    def one_step():
        qdist.broadcast_context(full_ctx, 0)
        ctx = qdist.shard_context(full_ctx, rank, world)
        out = loop.run(lat, ctx)
        return qdist.gather_latents(out, 0)

    def warm_eager():
        loop.set_inputs(lat, qdist.shard_context(full_ctx, rank, world))
        loop.step()

    dt, out = timed_steps(args, one_step, warm_eager, rank, world, dev, log)
    images = B * world * args.steps
    value = images / dt
    if rank == 0:
        assert out is not None and torch.isfinite(out.float()).all(), "non-finite latents"
        log(f"timed {args.steps} steps: {dt:.3f}s")
        int8 = args.mode.endswith("-int8")
        roof = dominant_kernel_roofline(dev, int8=int8)
        evals_per_s = value * args.denoise_steps  # UNet evals per image per step: 50 steps at CFG batch 2
        path_tflops = evals_per_s * 2 * UNET_GFLOP_PER_SAMPLE / 1e3
        t_min = int8_blended_tmin()
        wq = "W8A8" if args.mode.startswith("w8a8") else args.mode.upper()
        line = {
            "metric": f"images/sec SD1.5 {wq} {args.res}x{args.res} 50-step" + (" int8-MFMA" if int8 else ""),
            "value": round(value, 4), "unit": "images/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "i8 (int32 accumulate) + f16" if int8 else "f16",
            "data": "synthetic (random-init SD1.5 UNet weights N(0,1/fan_in), synthetic text embeddings and latents)",
            "config": {"workload": f"SD1.5 UNet {args.mode} {'int8-MFMA' if int8 else 'fake-quant'}, "
                                   f"{args.res}x{args.res}, {B} prompts/GPU "
                                   f"(CFG batch {2 * B}), {args.denoise_steps} DDIM steps, HIP graph per step",
                       "global_batch": B * world, "seq_len": 77, "parallelism": f"dp{world}"},
            "roofline": roof,
            "path_roofline": {"achieved": round(path_tflops / world, 1), "peak": PEAK_F16_TFLOPS,
                              "unit": "TFLOP/s per GPU", "frac": round(path_tflops / world / PEAK_F16_TFLOPS, 4),
                              "flop_per_image": 2 * args.denoise_steps * UNET_GFLOP_PER_SAMPLE * 1e9},
            "int8_blended_roofline": {"achieved": round(value / world, 4), "bound": round(1.0 / t_min, 2),
                                      "unit": "images/s per GPU", "frac": round(value / world * t_min, 4),
                                      "target_frac": 0.40,
                                      "basis": "67.72 TFLOP int8-eligible @ 5.0 POPS + 12.61 TFLOP attention @ 2.5 PF "
                                               "per 512^2 image (SURVEY 8d)"},
            "linear_kernel_choice": linear_families(),
        }
        if args.mode == "w4a16":
            line["weight_stream"] = weight_footprint(model)
        if not args.no_e2e:
            log("end to end (text encoder + VAE decode) ...")
            line["end_to_end"] = end_to_end(model, out[:B], prompts[:B], dt / args.steps)
    if world == 1 and not int8 and args.mode.startswith("w8a8") and not args.no_int8_mode:
        # north_star's target mode, measured in the same run: the same SD1.5 W8A8
        # workload quantized with int8_mfma=True, the same steps / warmup protocol
        line["int8_mode"] = int8_mode_line(args, dev, log, lat, full_ctx)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            line["cpu_baseline"] = cpu_baseline(args.cpu_threads or None)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def int8_blended_tmin():
    """Seconds per SD1.5 512^2 image at north_star's int8-blended bound of one GPU: the
    int8-eligible GEMM FLOP at the int8 peak + the attention FLOP at the fp16 peak."""
    return SD15_I8_FLOP_PER_IMAGE / (PEAK_I8_TOPS * 1e12) + SD15_F16_FLOP_PER_IMAGE / (PEAK_F16_TFLOPS * 1e12)


def timed_steps(args, one_step, warm_eager, rank, world, dev, log):
    """The bench contract's timing: W untimed warm-up steps, then exactly K steps bracketed by a
    barrier + device synchronize on both sides; the max over ranks.  Returns (seconds, last out)."""
    import torch
    import torch.distributed as dist
    from qdiff import dist as qdist
    if world > 1:
        qdist.share_gemm_table(warm_eager, rank, world)
    for _ in range(args.warmup):
        one_step()
    log("warmup done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item(), out


def int8_mode_line(args, dev, log, lat, full_ctx):
    """The int8-MFMA W8A8 mode (quantize(..., int8_mfma=True)) on the headline's
    workload and protocol (1 GPU): a second SD1.5 model built and calibrated like the first, its
    own 50-step graph loop over the same latents and text embeddings, timed over the same K steps
    after W warm-ups; with its int8-blended roofline fraction and the int8 dominant conv's
    roofline (HIP events live, PMC HBM traffic from the committed rocprofv3 pass)."""
    import torch
    import argparse as _ap
    a8 = _ap.Namespace(**vars(args))
    a8.mode = args.mode + "-int8"
    model = build_model(a8, dev)
    log(f"int8-MFMA model built + quantized ({a8.mode})")
    B = args.batch
    loop = model.get_loop(B, args.res, args.res, args.denoise_steps, 7.5, use_graph=True)
    from qdiff import dist as qdist
    ctx = qdist.shard_context(full_ctx, 0, 1)

    def one_step():
        return loop.run(lat, ctx)

    dt, out = timed_steps(a8, one_step, None, 0, 1, dev, log)
    assert out is not None and torch.isfinite(out.float()).all(), "non-finite int8-mode latents"
    value = B * args.steps / dt
    log(f"int8 mode: timed {args.steps} steps: {dt:.3f}s")
    t_min = int8_blended_tmin()
    return {"metric": f"images/sec SD1.5 W8A8 {args.res}x{args.res} 50-step int8-MFMA", "value": round(value, 4),
            "unit": "images/s", "ms_per_step": round(dt / args.steps * 1e3, 2), "steps": args.steps,
            "warmup": args.warmup, "dtype": "i8 (int32 accumulate) + f16",
            "config": f"same workload as the headline (SD1.5 {a8.mode}, {B} prompts, CFG batch {2 * B}, "
                      f"{args.denoise_steps} DDIM steps, HIP graph per step), quantize(..., int8_mfma=True)",
            "int8_blended_roofline": {"achieved": round(value, 4), "bound": round(1.0 / t_min, 2),
                                      "unit": "images/s per GPU", "frac": round(value * t_min, 4),
                                      "target_frac": 0.40},
            "roofline": dominant_kernel_roofline(dev, int8=True)}


def mmdit_dominant_roofline(model, dev, s, iters=10):
    """The largest GEMM class of the SD3.5 step: ff.net.0.proj of block 0 on the CFG batch's
    x-stream tokens (M = 2 S, N = 4C, K = C), through the same run_linear call the model makes
    (int4 codes or the tuned fp16 LDS-DMA family), timed with HIP events on its stream."""
    import torch
    from qdiff.unet import run_linear
    layer = model.pipeline.transformer.transformer_blocks[0].ff.net[0].proj
    k, n = layer.in_features, layer.out_features
    m = 2 * s
    x = torch.randn(m, k, generator=torch.Generator().manual_seed(0)).half().to(dev)
    for _ in range(3):
        run_linear(layer, x)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        run_linear(layer, x)
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tflops = 2.0 * m * n * k / (ms * 1e-3) / 1e12
    f8 = getattr(layer, "fp8_act", False)
    peak = PEAK_F8_TFLOPS if f8 else PEAK_F16_TFLOPS
    from qdiff import kernels as K
    ran = sorted({key[-1][ch[0]] for key, ch in K.gemm_choices().items()
                  if ch is not None and key[0] == "linear" and key[1:4] == (m, n, k)})
    return {"bound": "mfma", "achieved": round(tflops, 1), "peak": peak, "unit": "TFLOP/s",
            "frac": round(tflops / peak, 4), "traffic": None,
            "kernel": f"ff.net.0.proj GEMM M={m} N={n} K={k} "
                      + ("(e4m3 x e4m3, v_mfma_scale_f32_16x16x128_f8f6f4, per-token quant included)" if f8 else
                         f"({getattr(layer, 'qfmt', 'f16')} weights, {'/'.join(ran) or '?'} operand ran)"),
            "avg_us": round(ms * 1e3, 2)}


def cpu_baseline_sd35(threads, cfg, s, sc, steps):
    """The reference's CPU path for SD3.5 (torch-CPU fp16 F.linear / SDPA, the ops the fake-quant
    MMDiT runs) on a bounded sample: one FF-shaped linear over 256 tokens and one joint-attention
    head group, extrapolated by the analytic FLOPs of a 1024^2 image (GEMM vs attention)."""
    import torch
    import torch.nn.functional as F
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    c = cfg.inner_dim
    x = torch.randn(256, c, generator=g).half()
    w = (torch.randn(4 * c, c, generator=g) * 0.02).half()
    L = s + sc
    q = torch.randn(1, 2, L, cfg.attention_head_dim, generator=g).half()

    def med3(fn):  # the SD1.5 baseline's protocol (oracle/cpu_baseline.py): 1 warm-up + median of 3
        fn()
        ts = []
        for _ in range(3):
            t0 = time.time()
            fn()
            ts.append(time.time() - t0)
        return sorted(ts)[1]

    t_lin = med3(lambda: F.linear(x, w))
    lin_rate = 2 * 256 * 4 * c * c / t_lin
    t_att = med3(lambda: F.scaled_dot_product_attention(q, q, q))
    att_rate = 4 * 2 * L * L * cfg.attention_head_dim / t_att
    att_gflop = cfg.num_layers * 4 * L * L * c / 1e9
    gemm_gflop = mmdit_gflop_per_sample(cfg, s, sc) - att_gflop
    per_image = steps * 2 * (gemm_gflop * 1e9 / lin_rate + att_gflop * 1e9 / att_rate)
    return {"value": round(1.0 / per_image, 10), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": (f"fp16 linear {c}->{4 * c} x256 tokens {t_lin:.2f}s ({lin_rate / 1e9:.2f} GFLOP/s), SDPA "
                       f"2 heads x {L}^2 d{cfg.attention_head_dim} {t_att:.2f}s ({att_rate / 1e9:.2f} GFLOP/s); "
                       f"each 1 warm-up + median of 3; image = {steps} steps x CFG 2 x class FLOPs / class rates"),
            "seconds_per_image": round(per_image, 1)}


def main_sd35(args, model, rank, world, dev, log):
    """SD3.5-Large W4A16 g128 1024^2 (SURVEY config C5: batch 8 on 8 GPUs = 1 prompt per GPU)."""
    import torch
    import torch.distributed as dist
    from qdiff import dist as qdist
    from qdiff.pipeline import synthetic_text_embeddings
    cfg = model.pipeline.transformer.config
    B = args.batch
    hw = args.res // 8
    sc = 333
    s = (hw // cfg.patch_size) ** 2
    loop = model.get_loop(B, args.res, args.res, args.denoise_steps, 7.0, use_graph=True, ctx_len=sc)
    full_ctx = torch.empty(2 * B * world, sc, cfg.joint_attention_dim, dtype=torch.float16, device=dev)
    full_pooled = torch.empty(2 * B * world, cfg.pooled_projection_dim, dtype=torch.float16, device=dev)
    if rank == 0:
        prompts = [f"a photograph of synthetic scene {i}" for i in range(B * world)]
        negs = [""] * (B * world)
        full_ctx.copy_(torch.cat([synthetic_text_embeddings(negs, seq_len=sc, dim=cfg.joint_attention_dim, device=dev),
                                  synthetic_text_embeddings(prompts, seq_len=sc, dim=cfg.joint_attention_dim,
                                                            device=dev)]))
        full_pooled.copy_(torch.cat([
            synthetic_text_embeddings([f"{p}\x00pooled" for p in negs], seq_len=1, dim=cfg.pooled_projection_dim,
                                      device=dev)[:, 0],
            synthetic_text_embeddings([f"{p}\x00pooled" for p in prompts], seq_len=1, dim=cfg.pooled_projection_dim,
                                      device=dev)[:, 0]]))
    g = torch.Generator().manual_seed(42 + rank)
    lat = torch.randn(B, cfg.in_channels, hw, hw, generator=g).half().to(dev)

    def one_step():
        qdist.broadcast_context(full_ctx, 0)
        qdist.broadcast_context(full_pooled, 0)
        out = loop.run(lat, qdist.shard_context(full_ctx, rank, world), qdist.shard_context(full_pooled, rank, world))
        return qdist.gather_latents(out, 0)

    def warm_eager():
        loop.set_inputs(lat, qdist.shard_context(full_ctx, rank, world), qdist.shard_context(full_pooled, rank, world))
        loop.step()

    if world > 1:
        qdist.share_gemm_table(warm_eager, rank, world)
    for _ in range(args.warmup):
        one_step()
    log("warmup done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    value = B * world * args.steps / dt
    if rank == 0:
        assert out is not None and torch.isfinite(out.float()).all(), "non-finite latents"
        log(f"timed {args.steps} steps: {dt:.3f}s")
        gflop = mmdit_gflop_per_sample(cfg, s, sc)
        path_tflops = value * args.denoise_steps * 2 * gflop / 1e3
        line = {
            "metric": f"images/sec SD3.5-Large {args.mode.upper()} {args.res}x{args.res} {args.denoise_steps}-step",
            "value": round(value, 4), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "e4m3 activations x e4m3-coded W4 (fp32 accumulate) + f16" if args.mode == "w4a8-fp8" else "f16",
            "data": "synthetic (random-init SD3.5-Large MMDiT weights N(0,1/fan_in), synthetic text embeddings)",
            "config": {"workload": f"SD3.5-Large MMDiT {args.mode} g128 fake-quant, {args.res}x{args.res}, {B} "
                                   f"prompt(s)/GPU (CFG batch {2 * B}), {args.denoise_steps} flow-match Euler "
                                   f"steps, HIP graph per step (SURVEY config C5)",
                       "global_batch": B * world, "seq_len": sc, "parallelism": f"dp{world}"},
            "roofline": mmdit_dominant_roofline(model, dev, s),
            "path_roofline": {"achieved": round(path_tflops / world, 1), "peak": PEAK_F16_TFLOPS,
                              "unit": "TFLOP/s per GPU", "frac": round(path_tflops / world / PEAK_F16_TFLOPS, 4),
                              "flop_per_image": round(2 * args.denoise_steps * gflop * 1e9)},
            "linear_kernel_choice": linear_families(),
        }
        if args.mode == "w4a16":
            line["weight_stream"] = weight_footprint(model)
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            line["cpu_baseline"] = cpu_baseline_sd35(min(args.cpu_threads or 1 << 30, usable_cores()[0]), cfg, s, sc,
                                                     args.denoise_steps)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


SDXL_TFLOP_PER_SAMPLE = 6.76   # SDXL 1024^2 UNet eval, 88 % quantizable GEMM


def main_sdxl(args, model, rank, world, dev, log):
    """SDXL W8A8 1024^2 (SURVEY config C4: batch 16 on 8 GPUs = 2 prompts per GPU), 50
    EulerDiscrete steps at guidance 5.0, text_time conditioning, graph per step."""
    import torch
    import torch.distributed as dist
    from qdiff import dist as qdist
    from qdiff.pipeline import synthetic_text_embeddings
    cfg = model.pipeline.unet.config
    B = args.batch
    hw = args.res // 8
    pooled = cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim
    loop = model.get_loop(B, args.res, args.res, args.denoise_steps, 5.0, use_graph=True)
    full_ctx = torch.empty(2 * B * world, 77, cfg.cross_attention_dim, dtype=torch.float16, device=dev)
    full_text = torch.empty(2 * B * world, pooled, dtype=torch.float16, device=dev)
    if rank == 0:
        prompts = [f"a photograph of synthetic scene {i}" for i in range(B * world)]
        negs = [""] * (B * world)
        full_ctx.copy_(torch.cat([synthetic_text_embeddings(negs, dim=cfg.cross_attention_dim, device=dev),
                                  synthetic_text_embeddings(prompts, dim=cfg.cross_attention_dim, device=dev)]))
        full_text.copy_(torch.cat([
            synthetic_text_embeddings([f"{p}\x00pooled" for p in negs], seq_len=1, dim=pooled, device=dev)[:, 0],
            synthetic_text_embeddings([f"{p}\x00pooled" for p in prompts], seq_len=1, dim=pooled, device=dev)[:, 0]]))
    time_ids = torch.tensor([[args.res, args.res, 0, 0, args.res, args.res]] * (2 * B), dtype=torch.float32)
    g = torch.Generator().manual_seed(42 + rank)
    lat = torch.randn(B, 4, hw, hw, generator=g).half().to(dev)

    def one_step():
        qdist.broadcast_context(full_ctx, 0)
        qdist.broadcast_context(full_text, 0)
        out = loop.run(lat, qdist.shard_context(full_ctx, rank, world), qdist.shard_context(full_text, rank, world),
                       time_ids)
        return qdist.gather_latents(out, 0)

    def warm_eager():
        loop.set_inputs(lat, qdist.shard_context(full_ctx, rank, world), qdist.shard_context(full_text, rank, world),
                        time_ids)
        loop.step()

    if world > 1:
        qdist.share_gemm_table(warm_eager, rank, world)
    for _ in range(args.warmup):
        one_step()
    log("warmup done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    value = B * world * args.steps / dt
    if rank == 0:
        assert out is not None and torch.isfinite(out.float()).all(), "non-finite latents"
        log(f"timed {args.steps} steps: {dt:.3f}s")
        path_tflops = value * args.denoise_steps * 2 * SDXL_TFLOP_PER_SAMPLE
        line = {
            "metric": f"images/sec SDXL {args.mode.upper()} {args.res}x{args.res} {args.denoise_steps}-step",
            "value": round(value, 4), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f16",
            "data": "synthetic (random-init SDXL UNet weights N(0,1/fan_in), synthetic text embeddings and latents)",
            "config": {"workload": f"SDXL UNet {args.mode} fake-quant, {args.res}x{args.res}, {B} prompts/GPU "
                                   f"(CFG batch {2 * B}), {args.denoise_steps} EulerDiscrete steps, HIP graph per step "
                                   f"(SURVEY config C4)",
                       "global_batch": B * world, "seq_len": 77, "parallelism": f"dp{world}"},
            "roofline": dominant_kernel_roofline(dev, n=2 * B, h=hw, w=hw, c=cfg.block_out_channels[0]),
            "path_roofline": {"achieved": round(path_tflops / world, 1), "peak": PEAK_F16_TFLOPS,
                              "unit": "TFLOP/s per GPU", "frac": round(path_tflops / world / PEAK_F16_TFLOPS, 4),
                              "flop_per_image": round(2 * args.denoise_steps * SDXL_TFLOP_PER_SAMPLE * 1e12)},
        }
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            base = cpu_baseline(args.cpu_threads or None)
            # the SD1.5 C1 image's seconds scaled by the FLOP ratio of one SDXL image
            per_image = base["seconds_per_image"] * (2 * args.denoise_steps * SDXL_TFLOP_PER_SAMPLE * 1e12) / \
                (2 * 10 * UNET_GFLOP_PER_SAMPLE * 1e9)
            line["cpu_baseline"] = {"value": round(1.0 / per_image, 10), "unit": "images/s", "cores": base["cores"],
                                    "kind": "port", "sample": base["sample"] + "; scaled to one SDXL 1024^2 image by "
                                    "the FLOP ratio (6.76 TFLOP per SDXL eval vs 0.803 for SD1.5; 50 vs 10 steps)",
                                    "seconds_per_image": round(per_image, 1)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
