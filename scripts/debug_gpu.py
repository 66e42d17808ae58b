"""GPU debugging helper (not part of the product): NaN localisation in the full SD1.5 UNet and
DDIM-kernel intermediate dumps.  Writes gpurun_out/debug_*.npz / prints a report."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402
from qdiff import unet as U  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out")
os.makedirs(OUT, exist_ok=True)
dev = torch.device("cuda:0")


def ddim_dump():
    from oracle.unet_ref import ddim_step
    from qdiff.scheduler import ddim_tables
    ts, a_t, a_p = ddim_tables(50)
    g = torch.Generator().manual_seed(2)
    B, h, w = 2, 8, 8
    lat = torch.randn(B, 4, h, w, generator=g).half()
    eps = torch.randn(2 * B, 4, h, w, generator=g).half()
    lat_h = K.nchw_to_nhwc(lat.to(dev), 8)
    eps_h = K.nchw_to_nhwc(eps.to(dev), 8)
    nxt = torch.zeros(2 * B, h, w, 8, dtype=torch.float16, device=dev)
    step = torch.tensor([5], dtype=torch.int32, device=dev)
    K.cfg_ddim_step(lat_h, eps_h, 7.5, a_t.to(dev), a_p.to(dev), step, nxt, c=4)
    got = K.nhwc_to_nchw(lat_h, 4).cpu()
    ref = ddim_step(eps, 5, lat, a_t, a_p, 7.5)
    np.savez(os.path.join(OUT, "debug_ddim.npz"), lat=lat.numpy(), eps=eps.numpy(), got=got.numpy(), ref=ref.numpy(),
             a_t=a_t.numpy(), a_p=a_p.numpy(), lat_h=K.nhwc_to_nchw(lat_h, 4).cpu().numpy())
    print("ddim mismatches", int((got != ref).sum()), "max", (got.float() - ref.float()).abs().max().item())


def nan_hunt(mode):
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    qc = dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)
    if mode == "rtn":
        model.quantize(quant_config=qc, quantUnet=True)
    elif mode == "sq":
        model.quantize(quant_config=qc, quantType="sq", quantUnet=True,
                       calibration=dict(n_samples=2, batch_size=2, num_inference_steps=2))
        bad = [n for n, p in model.pipeline.unet.named_buffers() if not torch.isfinite(p.float()).all()]
        bad += [n for n, p in model.pipeline.unet.named_parameters() if not torch.isfinite(p.float()).all()]
        print("non-finite params/buffers after SQ:", bad[:10])
        for n, m in model.pipeline.unet.named_modules():
            if isinstance(m, torch.nn.LayerNorm) and ("norm1" in n or "norm3" in n):
                w = m.weight.float()
                print("LN", n, "min", w.abs().min().item(), "max", w.abs().max().item())
                break
    unet = model.pipeline.unet
    # instrument the block functions to report the first non-finite output
    first = []

    def wrap(fn, name):
        def f(*a, **k):
            out = fn(*a, **k)
            if not first and not torch.isfinite(out.float()).all():
                first.append(name)
                print("FIRST NON-FINITE after", name, "input finite:",
                      bool(torch.isfinite(a[1].float()).all()) if len(a) > 1 and torch.is_tensor(a[1]) else "?")
            return out
        return f

    for nm in ("resnet_fwd", "transformer_fwd", "block_fwd", "run_conv", "run_linear"):
        setattr(U, nm, wrap(getattr(U, nm), nm))
    g = torch.Generator().manual_seed(42)
    x = torch.randn(8, 4, 64, 64, generator=g).half()
    ctx = torch.randn(8, 77, 768, generator=g).half().to(dev)
    kv = unet.prepare_context(ctx)
    xh = K.nchw_to_nhwc(x.to(dev), 8)
    ts = torch.tensor([981.0], device=dev)
    temb = K.timestep_embedding(ts, None, 8, 320)
    out = unet.fwd(xh, temb, kv)
    torch.cuda.synchronize()
    print(mode, "finite:", bool(torch.isfinite(out.float()).all()), "std", out.float().std().item(), "first:", first)


def loop_hunt(mode, use_graph, steps=50):
    from qdiff.models import StableDiffusion1_x
    from qdiff.pipeline import synthetic_text_embeddings
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    qc = dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)
    if mode == "sq":
        model.quantize(quant_config=qc, quantType="sq", quantUnet=True,
                       calibration=dict(n_samples=4, batch_size=4, num_inference_steps=2))
    elif mode == "rtn":
        model.quantize(quant_config=qc, quantUnet=True)
    B = 4
    loop = model.get_loop(B, 512, 512, steps, 7.5, use_graph=use_graph)
    prompts = [f"a photograph of synthetic scene {i}" for i in range(B)]
    ctx = torch.cat([synthetic_text_embeddings([""] * B, device=dev), synthetic_text_embeddings(prompts, device=dev)])
    g = torch.Generator().manual_seed(42)
    lat = torch.randn(B, 4, 64, 64, generator=g).half().to(dev)
    if not use_graph:
        loop.set_inputs(lat, ctx)
        for i in range(steps):
            out = loop.step()
            torch.cuda.synchronize()
            fin_o = bool(torch.isfinite(out.float()).all())
            fin_l = bool(torch.isfinite(loop.lat.float()).all())
            print(f"{mode} eager step {i}: out finite {fin_o} absmax {out.float().abs().max().item():.3g} "
                  f"lat finite {fin_l} absmax {loop.lat.float().abs().max().item():.3g} idx {loop.step_idx.item()}")
            if not (fin_o and fin_l):
                break
    else:
        res = loop.run(lat, ctx)
        torch.cuda.synchronize()
        print(f"{mode} graph run: finite {bool(torch.isfinite(res.float()).all())} absmax {res.float().abs().max().item():.3g}")
        res2 = loop.run(lat, ctx)
        print(f"{mode} graph rerun equal: {torch.equal(res, res2)}")


def determinism():
    """Run each kernel family twice on identical inputs; report any bitwise difference."""
    g = torch.Generator().manual_seed(0)

    def twice(name, fn):
        a = fn()
        torch.cuda.synchronize()
        b = fn()
        torch.cuda.synchronize()
        same = torch.equal(a, b)
        print(f"determinism {name}: {'OK' if same else 'DIFF'}"
              + ("" if same else f" maxdiff {(a.float() - b.float()).abs().max().item():.4g} n={int((a != b).sum())}"))

    x = torch.randn(32768, 320, generator=g).half().to(dev)
    w = (torch.randn(2560, 320, generator=g) / 18).half().to(dev)
    twice("linear 32768x2560x320 f16", lambda: K.linear(x, w, "f16"))
    x2 = torch.randn(2048, 1280, generator=g).half().to(dev)
    w2 = (torch.randn(1280, 1280, generator=g) / 36).half().to(dev)
    twice("linear 2048x1280x1280 f16 (128x128 tile)", lambda: K.linear(x2, w2, "f16"))
    codes, scales, wdq = K.weight_quant(w2, 128, 8)
    twice("linear i8", lambda: K.linear(x2, codes, "i8", scales, 128))
    xc = torch.randn(8, 64, 64, 320, generator=g).half().to(dev)
    wc = (torch.randn(320, 3, 3, 320, generator=g) / 54).half().to(dev)
    am = torch.empty(8 * 320, dtype=torch.float32, device=dev)
    twice("conv 320 @64", lambda: K.conv2d_nhwc(xc, wc, 320, 1, 1, amax=am))
    xs = torch.randn(8, 16, 16, 1280, generator=g).half().to(dev)
    ws = (torch.randn(1280, 3, 3, 1280, generator=g) / 100).half().to(dev)
    am2 = torch.empty(8 * 1280, dtype=torch.float32, device=dev)
    twice("conv 1280 @16 (128x128)", lambda: K.conv2d_nhwc(xs, ws, 1280, 1, 1, amax=am2))
    q = torch.randn(8, 4096, 320, generator=g).half().to(dev)
    twice("attention 4096 d40", lambda: K.attention(q, q, q, 8))
    q2 = torch.randn(8, 256, 1280, generator=g).half().to(dev)
    kv = torch.randn(8, 77, 1280, generator=g).half().to(dev)
    twice("attention 256x77 d160", lambda: K.attention(q2, kv, kv, 8))
    gam = torch.ones(960, dtype=torch.float16, device=dev)
    bet = torch.zeros(960, dtype=torch.float16, device=dev)
    xg = torch.randn(8, 64, 64, 960, generator=g).half().to(dev)
    twice("groupnorm 960 @64 q8", lambda: K.groupnorm_nhwc(xg, 32, 1e-5, gam, bet, silu=True, q_bits=8))
    xl = torch.randn(32768, 320, generator=g).half().to(dev)
    twice("layernorm", lambda: K.layernorm(xl, 1e-5, gam[:320], bet[:320]))
    twice("act per-channel nhwc", lambda: K.act_fakequant(xc, "per_channel", 8, layout=K.NHWC))


def unet_determinism():
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    model.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    unet = model.pipeline.unet
    g = torch.Generator().manual_seed(42)
    x = torch.randn(8, 4, 64, 64, generator=g).half()
    ctx = torch.randn(8, 77, 768, generator=g).half().to(dev)
    kv = unet.prepare_context(ctx)
    xh = K.nchw_to_nhwc(x.to(dev), 8)
    ts = torch.tensor([981.0], device=dev)
    temb = K.timestep_embedding(ts, None, 8, 320)
    outs = []
    import qdiff.unet as UU
    trace = []
    orig = {n: getattr(UU, n) for n in ("resnet_fwd", "transformer_fwd", "run_conv", "run_linear")}
    for rep in range(2):
        rec = []
        for n, fn in orig.items():
            def mk(fn, n):
                def f(*a, **k):
                    o = fn(*a, **k)
                    rec.append((n, o.detach().clone()))
                    return o
                return f
            setattr(UU, n, mk(fn, n))
        outs.append(unet.fwd(xh, temb, kv).clone())
        torch.cuda.synchronize()
        trace.append(rec)
    for n, fn in orig.items():
        setattr(UU, n, fn)
    print("unet fwd deterministic:", torch.equal(outs[0], outs[1]))
    for i, ((n1, a), (n2, b)) in enumerate(zip(trace[0], trace[1])):
        if not torch.equal(a, b):
            print(f"first divergence at call {i} ({n1}) shape {tuple(a.shape)} maxdiff {(a.float()-b.float()).abs().max().item():.4g}")
            break


def graph_state():
    from qdiff.models import StableDiffusion1_x
    from qdiff.pipeline import synthetic_text_embeddings
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    model.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    B = 4
    steps = 3
    prompts = [f"a photograph of synthetic scene {i}" for i in range(B)]
    ctx = torch.cat([synthetic_text_embeddings([""] * B, device=dev), synthetic_text_embeddings(prompts, device=dev)])
    g = torch.Generator().manual_seed(42)
    lat = torch.randn(B, 4, 64, 64, generator=g).half().to(dev)
    e = model.get_loop(B, 512, 512, steps, 7.5, use_graph=False)
    E1 = e.run(lat, ctx).clone()
    E2 = e.run(lat, ctx).clone()
    gl = model.get_loop(B, 512, 512, steps, 7.5, use_graph=True)
    G1 = gl.run(lat, ctx).clone()
    G2 = gl.run(lat, ctx).clone()
    G3 = gl.run(lat, ctx).clone()
    E3 = e.run(lat, ctx).clone()
    f = lambda a, b: f"{torch.equal(a, b)} ({(a.float()-b.float()).abs().max().item():.3g})"
    print("E1==E2", f(E1, E2), "E1==G1", f(E1, G1), "G1==G2", f(G1, G2), "G2==G3", f(G2, G3), "E1==E3", f(E1, E3))
    # one step only, graph vs eager, from identical inputs
    gl.set_inputs(lat, ctx)
    gl.graph.replay()
    o_g = gl.last_out.clone()
    l_g = gl.lat.clone()
    e.set_inputs(lat, ctx)
    o_e = e.step().clone()
    print("1-step out eq", f(o_g, o_e), "lat eq", f(l_g, e.lat), "idx", gl.step_idx.item(), e.step_idx.item())


def graph_50():
    from qdiff.models import StableDiffusion1_x
    from qdiff.pipeline import synthetic_text_embeddings
    model = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    model.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    B, steps = 4, 50
    prompts = [f"a photograph of synthetic scene {i}" for i in range(B)]
    ctx = torch.cat([synthetic_text_embeddings([""] * B, device=dev), synthetic_text_embeddings(prompts, device=dev)])
    g = torch.Generator().manual_seed(42)
    lat = torch.randn(B, 4, 64, 64, generator=g).half().to(dev)
    e = model.get_loop(B, 512, 512, steps, 7.5, use_graph=False)
    gl = model.get_loop(B, 512, 512, steps, 7.5, use_graph=True)
    f = lambda a, b: f"{torch.equal(a, b)} ({(a.float()-b.float()).abs().max().item():.3g})"
    G1 = gl.run(lat, ctx).clone()
    G2 = gl.run(lat, ctx).clone()
    E1 = e.run(lat, ctx).clone()
    print("50 steps: G1==E1", f(G1, E1), "G2==E1", f(G2, E1), "G1==G2", f(G1, G2), flush=True)
    # which persistent buffer changed?  snapshot everything the graph reads
    snap = {}
    unet = model.pipeline.unet
    for n, b in list(unet.named_buffers()) + list(unet.named_parameters()):
        if b is not None:
            snap["p:" + n] = b.detach().clone()
    for n, m in unet.named_modules():
        c = getattr(m, "_qd_cache", None)
        if c is not None:
            snap["c:" + n] = c[1].clone()
    for key, (k, v) in gl.ctx_kv.items():
        snap[f"kv:{key}"] = torch.cat([k.flatten(), v.flatten()]).clone()
    gl.set_inputs(lat, ctx)
    G3 = gl.run(lat, ctx).clone()
    print("G3==G1 (before eager)", f(G3, G1), flush=True)
    E2 = e.run(lat, ctx).clone()
    changed = []
    for n, m in unet.named_modules():
        c = getattr(m, "_qd_cache", None)
        if c is not None and "c:" + n in snap and (c[1].data_ptr() != 0) and not torch.equal(c[1], snap["c:" + n]):
            changed.append("c:" + n)
    for n, b in list(unet.named_buffers()) + list(unet.named_parameters()):
        if b is not None and not torch.equal(b, snap["p:" + n]):
            changed.append("p:" + n)
    print("changed after eager run:", changed[:10], flush=True)
    G4 = gl.run(lat, ctx).clone()
    print("G4==G1 (after eager)", f(G4, G1), flush=True)
    # one replay vs one eager step from identical inputs: first differing arena buffer
    gl.set_inputs(lat, ctx)
    e.set_inputs(lat, ctx)
    gl.graph.replay()
    e.step()
    torch.cuda.synchronize()
    print("arena sizes", len(gl.arena.bufs), len(e.arena.bufs), "GB", gl.arena.nbytes() / 1e9, flush=True)
    for i, (a, b) in enumerate(zip(gl.arena.bufs, e.arena.bufs)):
        if not torch.equal(a, b):
            print(f"first differing arena buffer #{i} shape {tuple(a.shape)} dtype {a.dtype} "
                  f"graph finite {bool(torch.isfinite(a.float()).all())} eager finite {bool(torch.isfinite(b.float()).all())}",
                  flush=True)
            if i > 0:
                pa, pb = gl.arena.bufs[i - 1], e.arena.bufs[i - 1]
                print(f"  previous #{i-1} shape {tuple(pa.shape)} equal {torch.equal(pa, pb)}")
            break
    kv_ok = all(torch.equal(gl.ctx_kv[k][0], e.ctx_kv[k][0]) and torch.equal(gl.ctx_kv[k][1], e.ctx_kv[k][1]) for k in gl.ctx_kv)
    print("ctx_kv equal", kv_ok, "temb", torch.equal(gl.temb_in, e.temb_in))
    # step-by-step: graph replay vs eager from identical state
    gl.set_inputs(lat, ctx)
    e.set_inputs(lat, ctx)
    for i in range(steps):
        gl.graph.replay()
        oe = e.step()
        torch.cuda.synchronize()
        if not torch.equal(gl.lat, e.lat) or not torch.equal(gl.last_out, oe):
            print(f"diverge at step {i}: lat {f(gl.lat, e.lat)} out {f(gl.last_out, oe)} idx {gl.step_idx.item()} {e.step_idx.item()}",
                  flush=True)
            # which tensors differ: temb
            print("temb eq", f(gl.temb_in, e.temb_in), "next_in eq", f(gl.next_in, e.next_in))
            break
    else:
        print("step-by-step identical over", steps, "steps")


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "graph":
        graph_state()
    if what == "graph50":
        graph_50()
    if what in ("all", "det"):
        determinism()
        unet_determinism()
    if what in ("all", "ddim"):
        ddim_dump()
    if what in ("all", "nan"):
        for m in ["fp16", "rtn", "sq"]:
            nan_hunt(m)
    if what in ("all", "loop"):
        loop_hunt("rtn", False, 50)
        loop_hunt("rtn", True, 50)
        loop_hunt("sq", True, 50)
