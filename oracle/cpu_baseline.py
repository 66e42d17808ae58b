"""CPU baseline of the reference's fake-quant path - TEST / BASELINE
INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg; never part of the product).

C1 = SD1.5 UNet, W8 RTN fake-quant (quantize/quantizer.py "awq" diffusion branch: fp16 dequantized
weights, A16), 1 prompt at 512x512, 10 DDIM steps with CFG = 10 UNet evaluations at batch 2.  The
reference runs exactly torch-CPU fp16 ops (F.conv2d / F.linear in fake_quant.py:223,339 and the
diffusers UNet's group_norm / layer_norm / SDPA), which the oracle restates op for op
(oracle/unet_ref.py RefUNet, bit-exact per op to the reference's goldens).

A full C1 run is infeasible on the GPU box's host: its torch-CPU Half conv2d takes a scalar path
(~0.7 GFLOP/s measured there, vs ~316 GFLOP/s through oneDNN's fp16 kernels on this container's
AVX512-FP16 / AMX Xeon), so one UNet evaluation would take ~20 minutes.  Protocol used instead:
  1. census: the oracle's own forward at C1 shapes with shape-recording ops (no arithmetic) gives
     every (op, shape) of one UNet evaluation and its multiplicity;
  2. each distinct shape is timed with real torch-CPU fp16 ops on a bounded slice (batch / rows /
     query rows cut so a sample is ~`budget` FLOP), 1 warm-up + median of 3, and scaled to the full
     shape by its FLOP (norms: by element) count;
  3. seconds per image = 10 evaluations x sum(multiplicity x scaled time).
Elementwise ops (SiLU, adds, concat, nearest upsample, GELU) are not timed: the result is an
upper bound on the reference's CPU speed.
"""
import math
import os
import statistics
import time

import torch
import torch.nn.functional as F

F16 = torch.float16


class _CensusOps:
    """RefUNet op table that records (op, shapes) and returns zeros of the output shape."""

    def __init__(self):
        self.calls = []

    def linear(self, x, w, b=None):
        self.calls.append(("linear", (x.numel() // x.shape[-1], x.shape[-1], w.shape[0])))
        return torch.zeros(*x.shape[:-1], w.shape[0], dtype=F16)

    def conv2d(self, x, w, b=None, stride=1, padding=0):
        n, ci, h, wd = x.shape
        co, _, kh, kw = w.shape
        ho, wo = (h + 2 * padding - kh) // stride + 1, (wd + 2 * padding - kw) // stride + 1
        self.calls.append(("conv2d", (n, ci, h, wd, co, kh, stride, padding)))
        return torch.zeros(n, co, ho, wo, dtype=F16)

    def group_norm(self, x, g, w, b, eps):
        self.calls.append(("group_norm", (tuple(x.shape), g)))
        return torch.zeros_like(x)

    def layer_norm(self, x, shape, w, b, eps):
        self.calls.append(("layer_norm", (x.numel() // x.shape[-1], x.shape[-1])))
        return torch.zeros_like(x)

    def scaled_dot_product_attention(self, q, k, v, **kw):
        self.calls.append(("sdpa", (q.shape[0], q.shape[1], q.shape[2], k.shape[2], q.shape[3])))
        return torch.zeros_like(q)


def census(cfg_dict, shapes_sd, batch=2, res=512, ctx_len=77):
    """{(op, shape): count} of one UNet evaluation (the oracle's forward with recording ops)."""
    from .unet_ref import RefUNet
    ref = RefUNet(cfg_dict, shapes_sd, None)
    ops = _CensusOps()
    ref.ops = ops
    h = res // 8
    x = torch.zeros(batch, cfg_dict["in_channels"], h, h, dtype=F16)
    ctx = torch.zeros(batch, ctx_len, cfg_dict["cross_attention_dim"], dtype=F16)
    ref.forward(x, 981, ctx)
    out = {}
    for key in ops.calls:
        out[key] = out.get(key, 0) + 1
    return out


def _flops(op, s):
    if op == "linear":
        m, k, n = s
        return 2.0 * m * k * n
    if op == "conv2d":
        n, ci, h, w, co, k, st, p = s
        ho, wo = (h + 2 * p - k) // st + 1, (w + 2 * p - k) // st + 1
        return 2.0 * n * ho * wo * co * ci * k * k
    if op == "sdpa":
        b, hh, sq, skv, d = s
        return 4.0 * b * hh * sq * skv * d
    if op == "group_norm":
        return float(math.prod(s[0]))
    return float(s[0] * s[1])


def _sample(op, s, budget, g):
    """(callable on a bounded slice, scale = full work / sample work)."""
    full = _flops(op, s)
    if op == "linear":
        m, k, n = s
        ms = max(16, min(m, int(budget / (2.0 * k * n)) or 16))
        x = torch.randn(ms, k, generator=g).to(F16)
        w = (torch.randn(n, k, generator=g) / k ** 0.5).to(F16)
        b = torch.zeros(n, dtype=F16)
        return (lambda: F.linear(x, w, b)), full / (2.0 * ms * k * n)
    if op == "conv2d":
        n, ci, h, wd, co, k, st, p = s
        per_row = 2.0 * ((wd + 2 * p - k) // st + 1) * co * ci * k * k
        rows = max(1, min((h + 2 * p - k) // st + 1, int(budget / per_row)))
        hs = max(1, (rows - 1) * st + k - 2 * p)  # input rows giving `rows` output rows
        x = torch.randn(1, ci, hs, wd, generator=g).to(F16)
        w = (torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5).to(F16)
        b = torch.zeros(co, dtype=F16)
        sample = _flops("conv2d", (1, ci, hs, wd, co, k, st, p))
        return (lambda: F.conv2d(x, w, b, st, p)), full / sample
    if op == "sdpa":
        b, hh, sq, skv, d = s
        qs = max(16, min(sq, int(budget / (4.0 * skv * d))))
        q = torch.randn(1, 1, qs, d, generator=g).to(F16)
        kk = torch.randn(1, 1, skv, d, generator=g).to(F16)
        return (lambda: F.scaled_dot_product_attention(q, kk, kk)), full / (4.0 * qs * skv * d)
    if op == "group_norm":
        shape, groups = s
        x = torch.randn(1, *shape[1:], generator=g).to(F16)
        w, bb = torch.ones(shape[1], dtype=F16), torch.zeros(shape[1], dtype=F16)
        return (lambda: F.group_norm(x, groups, w, bb, 1e-5)), float(shape[0])
    m, c = s
    ms = max(16, min(m, 4096))
    x = torch.randn(ms, c, generator=g).to(F16)
    w, bb = torch.ones(c, dtype=F16), torch.zeros(c, dtype=F16)
    return (lambda: F.layer_norm(x, (c,), w, bb, 1e-5)), m / ms


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def c1_baseline(cfg_dict, shapes_sd, threads=None, budget=1.2e8, evals=10, batch=2, seed=0):
    """Seconds per C1 image (and details) of the reference's torch-CPU fp16 UNet path."""
    threads = threads or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    cen = census(cfg_dict, shapes_sd, batch=batch)
    per_class, t_eval = {}, 0.0
    t0 = time.time()
    with torch.no_grad():
        for (op, s), cnt in sorted(cen.items(), key=lambda kv: kv[0][0]):
            fn, scale = _sample(op, s, budget, g)
            fn()  # warm-up
            ts = []
            for _ in range(3):
                a = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - a)
            t = statistics.median(ts) * scale
            t_eval += cnt * t
            c = per_class.setdefault(op, [0, 0.0, 0.0])
            c[0] += cnt
            c[1] += cnt * t
            c[2] += cnt * _flops(op, s)
    wall = time.time() - t0
    s_img = evals * t_eval
    return {"seconds_per_image": s_img, "seconds_per_unet_eval": t_eval, "distinct_shapes": len(cen),
            "ops_per_eval": sum(cen.values()), "wall_s": wall, "threads": threads, "cpu": cpu_model(),
            "per_class": {k: {"calls": v[0], "ms_per_eval": round(v[1] * 1e3, 1),
                              "gflop_per_eval": round(v[2] / 1e9, 1) if k in ("linear", "conv2d", "sdpa") else None,
                              "gflops": round(v[2] / v[1] / 1e9, 2) if k in ("linear", "conv2d", "sdpa") else None}
                          for k, v in per_class.items()}}
