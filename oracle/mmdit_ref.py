"""CPU oracle of the fake-quantized SD3 / SD3.5 MMDiT denoising step (TEST INFRASTRUCTURE).

Consumes a flat diffusers-keyed state dict (SD3Transformer2DModel names) and a config dict,
quantizes the weights with the golden-pinned restatement (oracle/unet_ref.quantize_state_dict,
the reference's swap decisions of quantizer.py:491-533: Linear outputs whose child name contains
q_proj / k_proj / v_proj - in the MMDiT the add_{q,k,v}_proj context projections - get a
per-token output fake-quant, fake_quant.py:224), and runs the forward with torch-CPU fp16 ops in
diffusers' op order:

  PatchEmbed (conv p x p stride p, + cropped sincos pos_embed)
  CombinedTimestepTextProjEmbeddings (Timesteps(256) -> linear_1/SiLU/linear_2, + text_embedder)
  context_embedder
  JointTransformerBlock x L (AdaLayerNormZero on both streams - AdaLayerNormContinuous on the
    context of the last, context_pre_only block -, joint attention over [x; context] with
    RMSNorm(head_dim) qk-norm, gated residuals, GELU-tanh FeedForward)
  AdaLayerNormContinuous norm_out, proj_out, unpatchify
  CFG + FlowMatchEulerDiscreteScheduler.step (shift 3.0)

Parity status: the fake-quant math is PINNED (golden vectors from the reference module); the
MMDiT architecture and the flow-match scheduler are restated from diffusers' published
SD3Transformer2DModel / FlowMatchEulerDiscreteScheduler, which are not installed here -> that
part is UNPINNED.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import fake_quant_torch as FT
from .unet_ref import _Fp32Ops, quantize_state_dict, timestep_embedding

F16 = torch.float16


class _Fp32OpsMM(_Fp32Ops):
    @staticmethod
    def layer_norm(x, shape, w, b, eps):
        return F.layer_norm(x.float(), shape, None if w is None else w.float(), None if b is None else b.float(),
                            eps).half()

    @staticmethod
    def gelu_tanh(x):
        return F.gelu(x.float(), approximate="tanh").half()


class _HalfOpsMM:
    linear = staticmethod(F.linear)
    conv2d = staticmethod(F.conv2d)
    layer_norm = staticmethod(F.layer_norm)
    scaled_dot_product_attention = staticmethod(F.scaled_dot_product_attention)

    @staticmethod
    def gelu_tanh(x):
        return F.gelu(x, approximate="tanh")


# ------------------------------------------------------------------ scheduler
def flowmatch_tables(num_inference_steps, num_train_timesteps=1000, shift=3.0):
    """FlowMatchEulerDiscreteScheduler(shift).set_timesteps(n): (timesteps f32 [n], sigmas f32 [n+1])."""
    n_t = num_train_timesteps
    ts = np.linspace(1, n_t, n_t, dtype=np.float32)[::-1].copy()
    s = torch.from_numpy(ts).to(torch.float32) / n_t
    s = shift * s / (1 + (shift - 1) * s)
    sigma_max, sigma_min = s[0].item(), s[-1].item()
    t = np.linspace(sigma_max * n_t, sigma_min * n_t, num_inference_steps)
    sig = t / n_t
    sig = shift * sig / (1 + (shift - 1) * sig)
    sig = torch.from_numpy(sig).to(torch.float32)
    timesteps = sig * n_t
    return timesteps, torch.cat([sig, torch.zeros(1)])


def euler_step(noise_pred_cfg_in, i, latents, sigmas, guidance):
    """CFG combine + FlowMatchEulerDiscreteScheduler.step in diffusers' op order."""
    u, c = noise_pred_cfg_in.chunk(2)
    v = u + guidance * (c - u)
    sample = latents.to(torch.float32)
    prev = sample + (sigmas[i + 1] - sigmas[i]) * v
    return prev.to(v.dtype)


# ------------------------------------------------------------------ model
def crop_pos_embed(pos_embed, max_size, h, w):
    """PatchEmbed.cropped_pos_embed: centre crop of the [1, max*max, C] table -> [1, h*w, C]."""
    top, left = (max_size - h) // 2, (max_size - w) // 2
    c = pos_embed.shape[-1]
    sp = pos_embed.reshape(1, max_size, max_size, c)[:, top:top + h, left:left + w, :]
    return sp.reshape(1, -1, c)


class RefMMDiT:
    """variant "half": torch-CPU Half kernels (the reference's library calls); variant "fp32":
    GEMM / conv / norm / attention / GELU in fp32, rounded to fp16 once (see RefUNet)."""

    def __init__(self, cfg, sd, qc=None, variant="half", fp8=False):
        """fp8=True: the W4A8-fp8 mode (oracle/fp8_ref.py) on every linear the product runs it on
        (4-bit group-128 codes, K % 128 == 0, N % 8 == 0) when the call has >= 64 rows."""
        self.cfg = cfg
        self.ops = _Fp32OpsMM if variant == "fp32" else _HalfOpsMM
        sd = {k: v.detach().to("cpu", F16).contiguous() for k, v in sd.items()}
        self.f8 = {}
        if fp8:
            from . import fp8_ref as F8R
            g = qc.get("q_group_size", 128)
            for key, w in sd.items():
                if key.endswith(".weight") and w.dim() == 2 and qc["w_bit"] <= 4 and g == 128 and \
                        w.shape[1] % 128 == 0 and w.shape[0] % 8 == 0:
                    self.f8[key[: -len(".weight")]] = F8R.weight_codes(w, qc["w_bit"], 128)
        if qc is not None:
            self.sd, self.flags = quantize_state_dict(sd, qc)
        else:
            self.sd, self.flags = sd, {}

    # ---- layers
    def lin(self, name, x):
        f8 = self.f8.get(name)
        if f8 is not None and x.numel() // x.shape[-1] >= 64:
            from . import fp8_ref as F8R
            xq, sa = F8R.quant_rows_fp8(x.reshape(-1, x.shape[-1]))
            _, y, _ = F8R.linear_fp8(xq, sa, f8[0], f8[1], 128, self.sd.get(name + ".bias"))
            y = y.view(*x.shape[:-1], -1)
            f = self.flags.get(name)
            if f and f["out_quant"]:
                y = FT.per_token(y, f["a_bit"])
            return y
        y = self.ops.linear(x, self.sd[name + ".weight"], self.sd.get(name + ".bias"))
        f = self.flags.get(name)
        if f and f["out_quant"]:
            y = FT.per_token(y, f["a_bit"])
        return y

    def conv(self, name, x, stride, padding):
        f = self.flags.get(name)
        quant = f is not None and f["quant"]
        if quant:
            x = self._act(f, x)
        y = self.ops.conv2d(x, self.sd[name + ".weight"], self.sd.get(name + ".bias"), stride, padding)
        if quant:
            y = self._act(f, y)
        return y

    def _act(self, f, x):
        if f["act"] == "per_group":
            return FT.per_group(x, 1, f["a_bit"])
        return FT.ACT[f["act"]](x, f["a_bit"])

    def ln(self, x):
        return self.ops.layer_norm(x, (x.shape[-1],), None, None, 1e-6)

    def rms(self, name, x):
        """diffusers RMSNorm: x * rsqrt(mean(x.float()^2) + eps) (fp32), .to(fp16), * weight."""
        var = x.to(torch.float32).pow(2).mean(-1, keepdim=True)
        y = x * torch.rsqrt(var + 1e-6)
        return y.to(F16) * self.sd[name + ".weight"]

    def ff(self, p, x):
        return self.lin(p + ".net.2", self.ops.gelu_tanh(self.lin(p + ".net.0.proj", x)))

    # ---- blocks
    def attn(self, p, nx, nc, pre):
        b, s, _ = nx.shape
        heads = self.cfg["num_attention_heads"]
        d = self.cfg["attention_head_dim"]
        qk_norm = self.cfg.get("qk_norm") == "rms_norm"

        def heads_view(t):
            return t.view(b, -1, heads, d).transpose(1, 2)

        q = heads_view(self.lin(p + ".to_q", nx))
        k = heads_view(self.lin(p + ".to_k", nx))
        v = heads_view(self.lin(p + ".to_v", nx))
        if qk_norm:
            q, k = self.rms(p + ".norm_q", q), self.rms(p + ".norm_k", k)
        cq = heads_view(self.lin(p + ".add_q_proj", nc))
        ck = heads_view(self.lin(p + ".add_k_proj", nc))
        cv = heads_view(self.lin(p + ".add_v_proj", nc))
        if qk_norm:
            cq, ck = self.rms(p + ".norm_added_q", cq), self.rms(p + ".norm_added_k", ck)
        q, k, v = torch.cat([q, cq], 2), torch.cat([k, ck], 2), torch.cat([v, cv], 2)
        o = self.ops.scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False)
        o = o.transpose(1, 2).reshape(b, -1, heads * d).to(q.dtype)
        ho, co = o[:, :s], o[:, s:]
        co = None if pre else self.lin(p + ".to_add_out", co)
        return self.lin(p + ".to_out.0", ho), co

    def self_attn(self, p, nx):
        """diffusers Attention + AttnProcessor2_0 (MMDiT-X attn2): image tokens only."""
        b = nx.shape[0]
        heads = self.cfg["num_attention_heads"]
        d = self.cfg["attention_head_dim"]

        def heads_view(t):
            return t.view(b, -1, heads, d).transpose(1, 2)

        q = heads_view(self.lin(p + ".to_q", nx))
        k = heads_view(self.lin(p + ".to_k", nx))
        v = heads_view(self.lin(p + ".to_v", nx))
        if self.cfg.get("qk_norm") == "rms_norm":
            q, k = self.rms(p + ".norm_q", q), self.rms(p + ".norm_k", k)
        o = self.ops.scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False)
        o = o.transpose(1, 2).reshape(b, -1, heads * d).to(q.dtype)
        return self.lin(p + ".to_out.0", o)

    def block(self, i, h, ctx, temb_silu):
        """diffusers JointTransformerBlock.forward; blocks listed in dual_attention_layers
        (SD3.5-Medium MMDiT-X) take SD35AdaLayerNormZeroX's 9 chunks and the attn2 residual."""
        p = f"transformer_blocks.{i}"
        pre = i == self.cfg["num_layers"] - 1
        dual = i in tuple(self.cfg.get("dual_attention_layers") or ())
        e1 = self.lin(p + ".norm1.linear", temb_silu)
        if dual:
            sh_msa, sc_msa, g_msa, sh_mlp, sc_mlp, g_mlp, sh_msa2, sc_msa2, g_msa2 = e1.chunk(9, dim=1)
        else:
            sh_msa, sc_msa, g_msa, sh_mlp, sc_mlp, g_mlp = e1.chunk(6, dim=1)
        ln_h = self.ln(h)
        nh = ln_h * (1 + sc_msa[:, None]) + sh_msa[:, None]
        nh2 = ln_h * (1 + sc_msa2[:, None]) + sh_msa2[:, None] if dual else None
        e2 = self.lin(p + ".norm1_context.linear", temb_silu)
        if pre:
            cscale, cshift = e2.chunk(2, dim=1)
            nc = self.ln(ctx) * (1 + cscale)[:, None, :] + cshift[:, None, :]
        else:
            c_sh_msa, c_sc_msa, c_g_msa, c_sh_mlp, c_sc_mlp, c_g_mlp = e2.chunk(6, dim=1)
            nc = self.ln(ctx) * (1 + c_sc_msa[:, None]) + c_sh_msa[:, None]
        ao, co = self.attn(p + ".attn", nh, nc, pre)
        h = h + g_msa.unsqueeze(1) * ao
        if dual:
            h = h + g_msa2.unsqueeze(1) * self.self_attn(p + ".attn2", nh2)
        nh = self.ln(h) * (1 + sc_mlp[:, None]) + sh_mlp[:, None]
        h = h + g_mlp.unsqueeze(1) * self.ff(p + ".ff", nh)
        if pre:
            return None, h
        ctx = ctx + c_g_msa.unsqueeze(1) * co
        nc = self.ln(ctx) * (1 + c_sc_mlp[:, None]) + c_sh_mlp[:, None]
        ctx = ctx + c_g_mlp.unsqueeze(1) * self.ff(p + ".ff_context", nc)
        return ctx, h

    @torch.no_grad()
    def forward(self, x, t, enc, pooled):
        """x [2B, Cin, H, W] fp16, t float timestep, enc [2B, Sc, joint_attention_dim] fp16,
        pooled [2B, pooled_projection_dim] fp16 -> [2B, Cout, H, W] fp16."""
        cfg = self.cfg
        p = cfg["patch_size"]
        b, _, hh, ww = x.shape
        hp, wp = hh // p, ww // p
        h = self.conv("pos_embed.proj", x, p, 0).flatten(2).transpose(1, 2)
        pos = crop_pos_embed(self.sd["pos_embed.pos_embed"], cfg["pos_embed_max_size"], hp, wp)
        h = (h + pos).to(h.dtype)
        tproj = timestep_embedding(torch.full((b,), float(t), dtype=torch.float32), 256, True, 0).to(F16)
        temb = self.lin("time_text_embed.timestep_embedder.linear_2",
                        F.silu(self.lin("time_text_embed.timestep_embedder.linear_1", tproj)))
        pe = self.lin("time_text_embed.text_embedder.linear_2",
                      F.silu(self.lin("time_text_embed.text_embedder.linear_1", pooled)))
        temb = temb + pe
        ctx = self.lin("context_embedder", enc)
        temb_silu = F.silu(temb)
        for i in range(cfg["num_layers"]):
            ctx, h = self.block(i, h, ctx, temb_silu)
        scale, shift = self.lin("norm_out.linear", temb_silu).chunk(2, dim=1)
        h = self.ln(h) * (1 + scale)[:, None, :] + shift[:, None, :]
        h = self.lin("proj_out", h)
        co = cfg["out_channels"]
        h = h.reshape(b, hp, wp, p, p, co)
        h = torch.einsum("nhwpqc->nchpwq", h)
        return h.reshape(b, co, hp * p, wp * p)


@torch.no_grad()
def denoise(model, latents, enc, pooled, timesteps, sigmas, guidance=7.0, steps=None):
    """The SD3 pipeline loop on CPU: latents after `steps` flow-match Euler steps."""
    lat = latents.to(F16)
    n = len(timesteps) if steps is None else steps
    for i in range(n):
        x = torch.cat([lat] * 2)
        out = model.forward(x, float(timesteps[i]), enc, pooled)
        lat = euler_step(out, i, lat, sigmas, guidance)
    return lat
