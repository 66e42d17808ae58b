"""The denoising loop on device: CFG batch, UNet, DDIM step - one HIP graph per step.

Replaces the hot loop of diffusers ``StableDiffusionPipeline.__call__`` that the reference
enters through ``BaseAWQForDiffusion.generate`` (models/base.py:828-850): for t in timesteps:
UNet(cat([latents]*2), t, text_emb) -> CFG combine -> scheduler.step.

Device-resident state: latents (NHWC, channels padded 4 -> 8), the duplicated UNet input, the
per-step scheduler constants and a device step counter that the fused CFG+DDIM kernel
increments, so one captured graph is replayed ``num_inference_steps`` times with no host work
between steps.
"""
import gc
import zlib

import torch

from . import arena as A
from . import kernels as K
from .scheduler import (DDIMConfig, EulerDiscreteConfig, FlowMatchConfig, PNDMConfig, ddim_tables,
                        euler_discrete_tables, flowmatch_tables, pndm_tables)

C_PAD = 8


def synthetic_text_embeddings(prompts, seq_len=77, dim=768, device="cuda"):
    """Deterministic stand-in for the CLIP text encoder (out of scope): each prompt
    string seeds a CPU generator (crc32) that draws N(0,1) [seq_len, dim] fp16 features."""
    if isinstance(prompts, str):
        prompts = [prompts]
    embs = []
    for p in prompts:
        g = torch.Generator("cpu").manual_seed(zlib.crc32(p.encode()) & 0x7FFFFFFF)
        embs.append(torch.randn(seq_len, dim, generator=g))
    return torch.stack(embs).to(torch.float16).to(device)


class DenoiseLoop:
    """Static-shape denoising loop for a fixed (batch, resolution, steps)."""

    def __init__(self, unet, batch, height=512, width=512, num_inference_steps=50, guidance_scale=7.5,
                 device="cuda", use_graph=True, sched_cfg=DDIMConfig(), ctx_len=77):
        self.unet = unet
        self.B = batch
        self.h, self.w = height // 8, width // 8
        self.steps = num_inference_steps
        self.guidance = float(guidance_scale)
        self.device = torch.device(device)
        self.use_graph = use_graph
        cfg = unet.config
        self.c0 = cfg.block_out_channels[0]
        self.cin = cfg.in_channels
        ts, a_t, a_p = ddim_tables(num_inference_steps, sched_cfg)
        self.timesteps = ts
        self.ts_f32 = ts.to(torch.float32).to(self.device)
        self.a_t = a_t.to(self.device)
        self.a_p = a_p.to(self.device)
        f16 = dict(dtype=torch.float16, device=self.device)
        self.lat = torch.zeros(batch, self.h, self.w, C_PAD, **f16)
        self.next_in = torch.zeros(2 * batch, self.h, self.w, C_PAD, **f16)
        self.temb_in = torch.zeros(2 * batch, self.c0, **f16)
        self.step_idx = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.ctx = torch.zeros(2 * batch, ctx_len, cfg.cross_attention_dim, **f16)
        self.ctx_kv = None
        self.graph = None
        self.last_out = None
        self.arena = A.Arena()

    # ---------------------------------------------------------------- inputs
    @torch.no_grad()
    def set_inputs(self, latents, ctx):
        """latents [B, 4, h, w] fp16 (NCHW, like diffusers); ctx [2B, S, D] fp16 (uncond first)."""
        if latents.shape != (self.B, self.cin, self.h, self.w):
            raise ValueError(f"latents must be {(self.B, self.cin, self.h, self.w)}, got {tuple(latents.shape)}")
        if ctx.shape != self.ctx.shape:
            raise ValueError(f"context must be {tuple(self.ctx.shape)}, got {tuple(ctx.shape)}")
        lat = latents.to(device=self.device, dtype=torch.float16).contiguous()
        K.nchw_to_nhwc(lat, C_PAD, out=self.lat)
        K.nchw_to_nhwc(lat, C_PAD, out=self.next_in[: self.B])
        K.nchw_to_nhwc(lat, C_PAD, out=self.next_in[self.B:])
        self.ctx.copy_(ctx)
        self.step_idx.zero_()
        if self.ctx_kv is None:
            self.ctx_kv = self.unet.prepare_context(self.ctx)
        else:
            fresh = self.unet.prepare_context(self.ctx)
            for key, (k, v) in fresh.items():
                self.ctx_kv[key][0].copy_(k)
                self.ctx_kv[key][1].copy_(v)

    # ---------------------------------------------------------------- one step
    @torch.no_grad()
    def step(self, frozen=False):
        """One denoising step; every intermediate comes from the loop's static arena."""
        with A.using(self.arena, frozen=frozen):
            K.timestep_embedding(self.ts_f32, self.step_idx, 2 * self.B, self.c0, flip_sin_to_cos=True,
                                 shift=float(self.unet.config.freq_shift), out=self.temb_in)
            out = self.unet.fwd(self.next_in, self.temb_in, self.ctx_kv, temb_shared=True)
            K.cfg_ddim_step(self.lat, out, self.guidance, self.a_t, self.a_p, self.step_idx, self.next_in,
                            c=self.cin)
        self.last_out = out
        return out

    @torch.no_grad()
    def capture(self):
        """Warm up eagerly (allocations, weight caches), then capture one step into a graph."""
        if self.ctx_kv is None:
            raise RuntimeError("set_inputs() before capture()")
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self.step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        # A dead Python cycle that still owns a graph, stream or event (an earlier pipeline, say)
        # must not be finalised inside the capture: its destructor's HIP calls are illegal while
        # a stream is capturing and abort the process.  Collect now, and keep the collector off
        # until the capture has ended.
        gc.collect()
        g = torch.cuda.CUDAGraph()
        gc_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g):
                self.step(frozen=True)   # no allocation may happen inside the capture
        finally:
            if gc_on:
                gc.enable()
        self.graph = g

    @torch.no_grad()
    def run(self, latents=None, ctx=None):
        """Run all steps; returns the final latents [B, 4, h, w] fp16 (NCHW)."""
        if latents is not None:
            self.set_inputs(latents, ctx)
        if self.use_graph and self.graph is None:
            self.capture()
            if latents is not None:  # the warm-up step consumed the inputs: restage them
                self.set_inputs(latents, ctx)
        for _ in range(self.steps):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.step()
        return self.latents_nchw()

    def latents_nchw(self):
        return K.nhwc_to_nchw(self.lat, self.cin)


class PNDMDenoiseLoop(DenoiseLoop):
    """SD1.5 with its checkpoint's own PNDMScheduler (skip_prk_steps PLMS): S + 1 UNet
    evaluations, CFG + the linear-multistep step fused in one kernel whose noise-prediction history
    (4 slots) and step-1 restart sample stay on device; same one-graph-per-step replay."""

    def __init__(self, unet, batch, height=512, width=512, num_inference_steps=50, guidance_scale=7.5,
                 device="cuda", use_graph=True, sched_cfg=PNDMConfig(), ctx_len=77):
        super().__init__(unet, batch, height, width, num_inference_steps, guidance_scale, device, use_graph,
                         sched_cfg, ctx_len)
        ts, a_t, a_p = pndm_tables(num_inference_steps, sched_cfg)
        self.timesteps = ts
        self.ts_f32 = ts.to(torch.float32).to(self.device)
        self.a_t = a_t.to(self.device)
        self.a_p = a_p.to(self.device)
        self.steps = len(ts)
        self.ets = torch.zeros(4, *self.lat.shape, dtype=torch.float16, device=self.device)
        self.cur = torch.zeros_like(self.lat)

    @torch.no_grad()
    def step(self, frozen=False):
        with A.using(self.arena, frozen=frozen):
            K.timestep_embedding(self.ts_f32, self.step_idx, 2 * self.B, self.c0, flip_sin_to_cos=True,
                                 shift=float(self.unet.config.freq_shift), out=self.temb_in)
            out = self.unet.fwd(self.next_in, self.temb_in, self.ctx_kv, temb_shared=True)
            K.cfg_pndm_step(self.lat, out, self.guidance, self.a_t, self.a_p, self.step_idx, self.ets, self.cur,
                            self.next_in, c=self.cin)
        self.last_out = out
        return out


def make_loop(unet, batch, height, width, steps, guidance, device, use_graph, sched_cfg, ctx_len=77):
    """The UNet denoising loop of the pipeline's scheduler (DDIM or PNDM; SDXL's Euler loop is built
    by its adapter)."""
    cls = PNDMDenoiseLoop if isinstance(sched_cfg, PNDMConfig) else DenoiseLoop
    return cls(unet, batch, height, width, steps, guidance, device=device, use_graph=use_graph, sched_cfg=sched_cfg,
               ctx_len=ctx_len)


class FlowMatchDenoiseLoop(DenoiseLoop):
    """The SD3 / SD3.5 loop (diffusers StableDiffusion3Pipeline.__call__): for t in timesteps:
    transformer(cat([latents]*2), t, prompt_embeds, pooled) -> CFG -> FlowMatchEuler step, with
    the same device-resident, one-graph-per-step structure as DenoiseLoop.  Latents are NHWC
    with the transformer's 16 channels (no padding); context_embedder / text_embedder outputs
    are computed once per generate (step-invariant)."""

    def __init__(self, transformer, batch, height=1024, width=1024, num_inference_steps=28, guidance_scale=7.0,
                 device="cuda", use_graph=True, sched_cfg=FlowMatchConfig(), ctx_len=333):
        self.unet = transformer
        self.B = batch
        self.h, self.w = height // 8, width // 8
        self.steps = num_inference_steps
        self.guidance = float(guidance_scale)
        self.device = torch.device(device)
        self.use_graph = use_graph
        cfg = transformer.config
        self.cin = cfg.in_channels
        if self.cin % 8 or cfg.out_channels != self.cin:
            raise ValueError("the flow-match loop needs in_channels == out_channels, a multiple of 8")
        ts, sig = flowmatch_tables(num_inference_steps, sched_cfg)
        self.timesteps = ts
        self.ts_f32 = ts.to(self.device)
        self.sigmas = sig.to(self.device)
        f16 = dict(dtype=torch.float16, device=self.device)
        self.lat = torch.zeros(batch, self.h, self.w, self.cin, **f16)
        self.next_in = torch.zeros(2 * batch, self.h, self.w, self.cin, **f16)
        self.temb_in = torch.zeros(2 * batch, 256, **f16)
        self.step_idx = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.ctx = torch.zeros(2 * batch, ctx_len, cfg.joint_attention_dim, **f16)
        self.pooled = torch.zeros(2 * batch, cfg.pooled_projection_dim, **f16)
        self.ctx_kv = None
        self.graph = None
        self.last_out = None
        self.arena = A.Arena()

    @torch.no_grad()
    def set_inputs(self, latents, ctx, pooled=None):
        """latents [B, 16, h, w] fp16 NCHW; ctx [2B, Sc, 4096], pooled [2B, 2048] (uncond first)."""
        if latents.shape != (self.B, self.cin, self.h, self.w):
            raise ValueError(f"latents must be {(self.B, self.cin, self.h, self.w)}, got {tuple(latents.shape)}")
        if ctx.shape != self.ctx.shape:
            raise ValueError(f"context must be {tuple(self.ctx.shape)}, got {tuple(ctx.shape)}")
        if pooled is None or pooled.shape != self.pooled.shape:
            raise ValueError(f"pooled projections must be {tuple(self.pooled.shape)}")
        lat = latents.to(device=self.device, dtype=torch.float16).contiguous()
        K.nchw_to_nhwc(lat, self.cin, out=self.lat)
        K.nchw_to_nhwc(lat, self.cin, out=self.next_in[: self.B])
        K.nchw_to_nhwc(lat, self.cin, out=self.next_in[self.B:])
        self.ctx.copy_(ctx)
        self.pooled.copy_(pooled)
        self.step_idx.zero_()
        fresh = self.unet.prepare_context(self.ctx, self.pooled)
        if self.ctx_kv is None:
            self.ctx_kv = fresh
        else:
            for key, t in fresh.items():
                self.ctx_kv[key].copy_(t)

    @torch.no_grad()
    def step(self, frozen=False):
        with A.using(self.arena, frozen=frozen):
            K.timestep_embedding(self.ts_f32, self.step_idx, 2 * self.B, 256, flip_sin_to_cos=True, shift=0.0,
                                 out=self.temb_in)
            out = self.unet.fwd(self.next_in, self.temb_in, self.ctx_kv)
            K.cfg_euler_step(self.lat, out, self.guidance, self.sigmas, self.step_idx, self.next_in)
        self.last_out = out
        return out

    @torch.no_grad()
    def run(self, latents=None, ctx=None, pooled=None):
        if latents is not None:
            self.set_inputs(latents, ctx, pooled)
        if self.use_graph and self.graph is None:
            self.capture()
            if latents is not None:
                self.set_inputs(latents, ctx, pooled)
        for _ in range(self.steps):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.step()
        return self.latents_nchw()


class EulerDiscreteDenoiseLoop(DenoiseLoop):
    """The SDXL loop (diffusers StableDiffusionXLPipeline.__call__ with its EulerDiscreteScheduler):
    latents * init_noise_sigma, then per step scale_model_input (x / sqrt(sigma^2 + 1)) ->
    UNet(x, t, prompt_embeds, added_cond_kwargs={text_embeds, time_ids}) -> CFG -> Euler step.
    The additional "text_time" embedding input [text_embeds | Timesteps(time_ids)] is
    step-invariant and built once per generate on device."""

    def __init__(self, unet, batch, height=1024, width=1024, num_inference_steps=50, guidance_scale=5.0,
                 device="cuda", use_graph=True, sched_cfg=EulerDiscreteConfig(), ctx_len=77):
        super().__init__(unet, batch, height, width, num_inference_steps, guidance_scale, device, use_graph,
                         sched_cfg, ctx_len)
        cfg = unet.config
        if cfg.addition_embed_type != "text_time":
            raise ValueError("the SDXL loop needs a UNet with addition_embed_type='text_time'")
        ts, sig, dsc, init = euler_discrete_tables(num_inference_steps, sched_cfg)
        self.timesteps = ts
        self.ts_f32 = ts.to(self.device)
        self.sigmas = sig.to(self.device)
        self.dscale = dsc.to(self.device)
        self.dscale0 = float(dsc[0])
        self.init_sigma = float(init)
        self.time_dim = cfg.addition_time_embed_dim
        self.text_dim = cfg.projection_class_embeddings_input_dim - 6 * self.time_dim
        f16 = dict(dtype=torch.float16, device=self.device)
        self.add_emb = torch.zeros(2 * batch, cfg.projection_class_embeddings_input_dim, **f16)

    @torch.no_grad()
    def set_inputs(self, latents, ctx, text_embeds=None, time_ids=None):
        """latents [B, 4, h, w]; ctx [2B, 77, D]; text_embeds [2B, pooled dim]; time_ids [2B, 6]
        (uncond first, as diffusers concatenates them)."""
        if latents.shape != (self.B, self.cin, self.h, self.w):
            raise ValueError(f"latents must be {(self.B, self.cin, self.h, self.w)}, got {tuple(latents.shape)}")
        if ctx.shape != self.ctx.shape:
            raise ValueError(f"context must be {tuple(self.ctx.shape)}, got {tuple(ctx.shape)}")
        if text_embeds is None or tuple(text_embeds.shape) != (2 * self.B, self.text_dim):
            raise ValueError(f"text_embeds must be {(2 * self.B, self.text_dim)}")
        if time_ids is None or tuple(time_ids.shape) != (2 * self.B, 6):
            raise ValueError(f"time_ids must be {(2 * self.B, 6)}")
        lat = latents.to(device=self.device, dtype=torch.float16).contiguous()
        K.nchw_to_nhwc(lat, C_PAD, out=self.lat)
        K.scale_latents(self.lat, self.init_sigma, self.dscale0, next_in=self.next_in, c=self.cin)
        self.ctx.copy_(ctx)
        tid = time_ids.to(device=self.device, dtype=torch.float32).reshape(-1).contiguous()
        temb = K.timestep_embedding(tid, None, tid.numel(), self.time_dim, flip_sin_to_cos=self.unet.config.flip_sin_to_cos,
                                    shift=float(self.unet.config.freq_shift), per_row=True)
        te = text_embeds.to(device=self.device, dtype=torch.float16).contiguous()
        K.concat_c(te, temb.view(2 * self.B, 6 * self.time_dim), out=self.add_emb)
        self.step_idx.zero_()
        fresh = self.unet.prepare_context(self.ctx)
        if self.ctx_kv is None:
            self.ctx_kv = fresh
        else:
            for key, (k, v) in fresh.items():
                self.ctx_kv[key][0].copy_(k)
                self.ctx_kv[key][1].copy_(v)

    @torch.no_grad()
    def step(self, frozen=False):
        with A.using(self.arena, frozen=frozen):
            K.timestep_embedding(self.ts_f32, self.step_idx, 2 * self.B, self.c0, flip_sin_to_cos=True,
                                 shift=float(self.unet.config.freq_shift), out=self.temb_in)
            out = self.unet.fwd(self.next_in, self.temb_in, self.ctx_kv, add_emb_in=self.add_emb)
            K.cfg_euler_discrete_step(self.lat, out, self.guidance, self.sigmas, self.dscale, self.step_idx,
                                      self.next_in, c=self.cin)
        self.last_out = out
        return out

    @torch.no_grad()
    def run(self, latents=None, ctx=None, text_embeds=None, time_ids=None):
        if latents is not None:
            self.set_inputs(latents, ctx, text_embeds, time_ids)
        if self.use_graph and self.graph is None:
            self.capture()
            if latents is not None:
                self.set_inputs(latents, ctx, text_embeds, time_ids)
        for _ in range(self.steps):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.step()
        return self.latents_nchw()
