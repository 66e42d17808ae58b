"""CPU oracle of the fake-quantized SD UNet denoising step (TEST INFRASTRUCTURE / CPU BASELINE).

Independent of the product package: it consumes a flat diffusers-keyed state dict and a config
dict, quantizes the weights with the golden-pinned numpy restatement (oracle/fake_quant_np.py)
following the reference's diffusion swap decisions (quantizer.py:491-533), and runs the
forward with torch-CPU fp16 NCHW ops in diffusers' op order - the same library calls the
reference makes through diffusers (F.conv2d / F.linear from fake_quant.py:223,339, group_norm,
layer_norm, SDPA, GEGLU, SiLU, nearest interpolate).

Parity status: the fake-quant math is PINNED (golden vectors from the reference module); the
UNet architecture/op order is restated from diffusers' published UNet2DConditionModel, which is
not installed here -> that part is UNPINNED.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import fake_quant_np as FQ
from . import fake_quant_torch as FT
from . import int8_ref as I8

I8_MIN_ROWS = 64  # the product's rule: linears with fewer input rows keep the fp16 MFMA (unet.py)

F16 = torch.float16


# ------------------------------------------------------------------ weight quantization
def quantize_state_dict(sd, qc, backend="torch", skip=()):
    """Return (qsd, flags): fake-quantized fp16 weights and per-layer activation flags.

    qc keys (AwqConfig): w_bit, a_bit, q_group_size, weight_quant_type, weight_quant_conv_type,
    act_quant_conv_type, quantize_act.  Linear = 2-D weight, Conv2d = 4-D weight.
    backend "torch" (fast, CPU fp16 ops) or "numpy"; both are pinned bit-exactly by the goldens.
    """
    if backend == "numpy":
        wq = {"group": lambda w, b, g: torch.from_numpy(np.ascontiguousarray(FQ.quantize_weight_absmax(w.numpy(), b, g))),
              "per_channel": lambda w, b: torch.from_numpy(np.ascontiguousarray(FQ.quantize_weight_per_channel_absmax(w.numpy(), b))),
              "per_tensor": lambda w, b: torch.from_numpy(np.ascontiguousarray(FQ.quantize_weight_per_tensor_absmax(w.numpy(), b)))}
    else:
        wq = {"group": FT.weight_group, "per_channel": FT.weight_per_channel, "per_tensor": FT.weight_per_tensor}
    qsd = dict(sd)
    flags = {}
    for key, w in sd.items():
        if not key.endswith(".weight") or w.dim() not in (2, 4):
            continue
        name = key[: -len(".weight")]
        child = name.split(".")[-1]
        if name in skip:  # int8-mode layer: its weight is already the per-channel int8 dequant
            if w.dim() == 2:
                flags[name] = {"kind": "linear", "out_quant": "k_proj" in child or "v_proj" in child or
                               "q_proj" in child, "a_bit": qc["a_bit"]}
            else:
                flags[name] = {"kind": "conv", "act": qc.get("act_quant_conv_type", "per_channel"), "quant": False,
                               "a_bit": qc["a_bit"]}
            continue
        w = w.to(F16).contiguous()
        if w.dim() == 2:
            wt = qc.get("weight_quant_type", "group")
            if wt == "group":
                q = wq["group"](w, qc["w_bit"], qc.get("q_group_size", 128))
            elif wt in ("per_channel", "per_tensor"):
                q = wq[wt](w, qc["w_bit"])
            else:
                raise ValueError(wt)
            qout = "k_proj" in child or "v_proj" in child or "q_proj" in child
            flags[name] = {"kind": "linear", "out_quant": qout, "a_bit": qc["a_bit"]}
        else:
            wt = qc.get("weight_quant_conv_type", "per_channel")
            if wt not in ("per_channel", "per_tensor"):
                raise ValueError(wt)
            q = wq[wt](w, qc["w_bit"])
            flags[name] = {"kind": "conv", "act": qc.get("act_quant_conv_type", "per_channel"),
                           "quant": bool(qc.get("quantize_act", False)), "a_bit": qc["a_bit"]}
        qsd[key] = q.contiguous()
    return qsd, flags


# ------------------------------------------------------------------ diffusers ops
def timestep_embedding(t, dim, flip_sin_to_cos=True, shift=0.0, max_period=10000):
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32)
    exponent = exponent / (half - shift)
    emb = torch.exp(exponent)
    emb = t[:, None].float() * emb[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


class _Fp32Ops:
    """Each torch op evaluated in fp32 and rounded to fp16 once ("single rounding" variant)."""

    @staticmethod
    def linear(x, w, b=None):
        return F.linear(x.float(), w.float(), None if b is None else b.float()).half()

    @staticmethod
    def conv2d(x, w, b=None, stride=1, padding=0):
        return F.conv2d(x.float(), w.float(), None if b is None else b.float(), stride, padding).half()

    @staticmethod
    def group_norm(x, g, w, b, eps):
        return F.group_norm(x.float(), g, w.float(), b.float(), eps).half()

    @staticmethod
    def layer_norm(x, shape, w, b, eps):
        return F.layer_norm(x.float(), shape, w.float(), b.float(), eps).half()

    @staticmethod
    def scaled_dot_product_attention(q, k, v, **kw):
        return F.scaled_dot_product_attention(q.float(), k.float(), v.float(), **kw).half()


class RefUNet:
    """variant "half": torch-CPU Half kernels, the reference's own library calls (default).
    variant "fp32": every GEMM / conv / norm / attention op computed in fp32 and rounded to fp16
    once - the same math with a single rounding per op, i.e. what an fp32-accumulating
    implementation (MFMA) computes.  The spread between the two variants measures how much the
    fake-quant network amplifies ulp-level differences (tests/test_gpu_unet.py)."""

    def __init__(self, cfg, sd, qc=None, variant="half", int8=False):
        """cfg: dict of UNetConfig fields; sd: {key: fp16 cpu tensor}; qc: AwqConfig dict or None.
        int8=True: the int8-MFMA W8A8 mode (oracle/int8_ref.py) on every eligible layer."""
        self.cfg = cfg
        self.ops = _Fp32Ops if variant == "fp32" else F
        sd = {k: v.detach().to("cpu", F16).contiguous() for k, v in sd.items()}
        self.i8 = {}
        if int8:
            sd = self._int8_weights(sd)
        if qc is not None:
            self.sd, self.flags = quantize_state_dict(sd, qc, skip=set(self.i8))
        else:
            self.sd, self.flags = sd, {}
        for name in self.i8:
            self.flags[name] = dict(self.flags.get(name, {}), int8=True)
        self.hooks = None  # optional {linear name: callable(x)} for calibration
        # optional {layer name: (input, output)} of every conv / linear / norm / SDPA call:
        # the teacher-forced per-layer parity test feeds each GPU layer these inputs
        self.record = None

    def _rec(self, name, *tensors):
        if self.record is not None:
            self.record[name] = tuple(t.detach().clone() for t in tensors)

    def _int8_weights(self, sd):
        """Per-output-channel int8 codes of every eligible layer (the product's rule: linear
        K % 64 == 0; conv Ci_pad % 64 == 0 and Co % 8 == 0); the state dict gets their
        dequantized values (the buffers the product's modules hold in this mode)."""
        out = dict(sd)
        for key, w in sd.items():
            if not key.endswith(".weight") or w.dim() not in (2, 4):
                continue
            name = key[: -len(".weight")]
            if w.dim() == 2:
                if w.shape[1] % 64:
                    continue
                q, sc = I8.weight_rows_i8(w.numpy())
                self.i8[name] = ("linear", q, sc)
                out[key] = torch.from_numpy(I8.weight_rows_dequant(w.numpy()))
            else:
                co, ci, kh, kw = w.shape
                if ((ci + 7) // 8 * 8) % 64 or co % 8:
                    continue
                wk = w.numpy().transpose(0, 2, 3, 1).reshape(co, -1)
                q, sc = I8.weight_rows_i8(wk)
                deq = I8.weight_rows_dequant(wk).reshape(co, kh, kw, ci)
                self.i8[name] = ("conv", q.reshape(co, kh, kw, ci).transpose(0, 3, 1, 2).copy(), sc)
                out[key] = torch.from_numpy(deq.transpose(0, 3, 1, 2).copy())
        return out

    # ---- layers
    def lin(self, name, x):
        if self.hooks is not None and name in self.hooks:
            self.hooks[name](x)
        i8 = self.i8.get(name)
        if i8 is not None and x.numel() // x.shape[-1] >= I8_MIN_ROWS:
            x2 = x.reshape(-1, x.shape[-1]).numpy()
            xq, sa = I8.quant_rows_i8(x2)
            b = self.sd.get(name + ".bias")
            y = torch.from_numpy(I8.linear_i8(xq, sa, i8[1], i8[2], None if b is None else b.numpy()))
            y = y.view(*x.shape[:-1], -1)
            f = self.flags.get(name)
            if f and f.get("out_quant"):
                y = FT.per_token(y, f["a_bit"])
            self._rec(name, x, y)
            return y
        y = self.ops.linear(x, self.sd[name + ".weight"], self.sd.get(name + ".bias"))
        f = self.flags.get(name)
        if f and f["out_quant"]:
            y = FT.per_token(y, f["a_bit"])
        self._rec(name, x, y)
        return y

    def conv(self, name, x, stride=1, padding=None):
        w = self.sd[name + ".weight"]
        if padding is None:
            padding = w.shape[-1] // 2
        i8 = self.i8.get(name)
        if i8 is not None:
            xq, sa = I8.quant_samples_i8(x.numpy())
            b = self.sd.get(name + ".bias")
            y = torch.from_numpy(I8.conv2d_i8(xq, sa, i8[1], i8[2], None if b is None else b.numpy(), stride, padding))
            self._rec(name, x, y)
            return y
        f = self.flags.get(name)
        quant = f is not None and f["quant"]
        x_in = x
        if quant:
            x = self._act(f, x)
        y = self.ops.conv2d(x, w, self.sd.get(name + ".bias"), stride, padding)
        if quant:
            y = self._act(f, y)
        self._rec(name, x_in, y)
        return y

    def _act(self, f, x):
        if f["act"] == "per_group":
            return FT.per_group(x, 1, f["a_bit"])
        return FT.ACT[f["act"]](x, f["a_bit"])

    def gn(self, name, x, groups, eps):
        y = self.ops.group_norm(x, groups, self.sd[name + ".weight"], self.sd[name + ".bias"], eps)
        self._rec(name, x, y)
        return y

    def ln(self, name, x):
        y = self.ops.layer_norm(x, (x.shape[-1],), self.sd[name + ".weight"], self.sd[name + ".bias"], 1e-5)
        self._rec(name, x, y)
        return y

    # ---- blocks
    def resnet(self, p, x, temb):
        g, eps = self.cfg["norm_num_groups"], self.cfg["norm_eps"]
        h = F.silu(self.gn(p + ".norm1", x, g, eps))
        h = self.conv(p + ".conv1", h)
        t = self.lin(p + ".time_emb_proj", F.silu(temb))[:, :, None, None]
        h = h + t
        h = F.silu(self.gn(p + ".norm2", h, g, eps))
        h = self.conv(p + ".conv2", h)
        if p + ".conv_shortcut.weight" in self.sd:
            x = self.conv(p + ".conv_shortcut", x)
        return x + h

    def attention(self, p, x, ctx, heads):
        q = self.lin(p + ".to_q", x)
        k = self.lin(p + ".to_k", ctx)
        v = self.lin(p + ".to_v", ctx)
        b = x.shape[0]
        d = q.shape[-1] // heads
        q = q.view(b, -1, heads, d).transpose(1, 2)
        k = k.view(b, -1, heads, d).transpose(1, 2)
        v = v.view(b, -1, heads, d).transpose(1, 2)
        o = self.ops.scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False)
        o = o.transpose(1, 2).reshape(b, -1, heads * d).to(q.dtype)
        if self.record is not None:
            self._rec(p + ".sdpa", q.transpose(1, 2).reshape(b, -1, heads * d), k.transpose(1, 2).reshape(b, -1, heads * d),
                      v.transpose(1, 2).reshape(b, -1, heads * d), o)
        return self.lin(p + ".to_out.0", o)

    def block(self, p, t, ctx, heads):
        n = self.ln(p + ".norm1", t)
        t = self.attention(p + ".attn1", n, n, heads) + t
        n = self.ln(p + ".norm2", t)
        t = self.attention(p + ".attn2", n, ctx, heads) + t
        n = self.ln(p + ".norm3", t)
        h, gate = self.lin(p + ".ff.net.0.proj", n).chunk(2, dim=-1)
        return self.lin(p + ".ff.net.2", h * F.gelu(gate)) + t

    def transformer(self, p, x, ctx, heads, layers):
        b, c, hh, ww = x.shape
        res = x
        h = self.gn(p + ".norm", x, self.cfg["norm_num_groups"], 1e-6)
        if self.cfg.get("use_linear_projection"):
            h = h.permute(0, 2, 3, 1).reshape(b, hh * ww, c)
            h = self.lin(p + ".proj_in", h)
        else:
            h = self.conv(p + ".proj_in", h)
            h = h.permute(0, 2, 3, 1).reshape(b, hh * ww, c)
        for i in range(layers):
            h = self.block(f"{p}.transformer_blocks.{i}", h, ctx, heads)
        if self.cfg.get("use_linear_projection"):
            h = self.lin(p + ".proj_out", h)
            h = h.reshape(b, hh, ww, c).permute(0, 3, 1, 2).contiguous()
        else:
            h = h.reshape(b, hh, ww, c).permute(0, 3, 1, 2).contiguous()
            h = self.conv(p + ".proj_out", h)
        return h + res

    def _heads(self, i):
        h = self.cfg["attention_head_dim"]
        return h[i] if isinstance(h, (list, tuple)) else h

    def _layers(self, i):
        t = self.cfg.get("transformer_layers_per_block", 1)
        return t[i] if isinstance(t, (list, tuple)) else t

    def add_embeds(self, text_embeds, time_ids):
        """SDXL "text_time" conditioning input (UNet2DConditionModel.get_aug_embed): Timesteps of
        the flattened time_ids (fp32), reshaped per sample, concatenated after the pooled text
        embeddings (fp16 | fp32 -> fp32) and cast to fp16."""
        cfg = self.cfg
        te = timestep_embedding(time_ids.flatten().float(), cfg["addition_time_embed_dim"],
                                cfg.get("flip_sin_to_cos", True), cfg.get("freq_shift", 0))
        te = te.reshape(text_embeds.shape[0], -1)
        return torch.cat([text_embeds, te], dim=-1).to(F16)

    @torch.no_grad()
    def forward(self, x, t, ctx, add_emb=None):
        """x [2B, 4, h, w] fp16, t timestep (int; float for the Euler scheduler), ctx [2B, S, D]
        fp16, add_emb [2B, P] fp16 (SDXL add_embeds) -> eps [2B, 4, h, w] fp16."""
        cfg = self.cfg
        ch = cfg["block_out_channels"]
        b = x.shape[0]
        tt = torch.full((b,), t, dtype=torch.float32 if isinstance(t, float) else torch.int64)
        temb = timestep_embedding(tt, ch[0], cfg.get("flip_sin_to_cos", True), cfg.get("freq_shift", 0)).to(F16)
        temb = self.lin("time_embedding.linear_2", F.silu(self.lin("time_embedding.linear_1", temb)))
        if cfg.get("addition_embed_type") == "text_time":
            aug = self.lin("add_embedding.linear_2", F.silu(self.lin("add_embedding.linear_1", add_emb)))
            temb = temb + aug
        h = self.conv("conv_in", x)
        skips = [h]
        nlev = len(ch)
        for i, typ in enumerate(cfg["down_block_types"]):
            for j in range(cfg["layers_per_block"]):
                h = self.resnet(f"down_blocks.{i}.resnets.{j}", h, temb)
                if typ == "CrossAttnDownBlock2D":
                    h = self.transformer(f"down_blocks.{i}.attentions.{j}", h, ctx, self._heads(i), self._layers(i))
                skips.append(h)
            if i < nlev - 1:
                h = self.conv(f"down_blocks.{i}.downsamplers.0.conv", h, stride=2, padding=1)
                skips.append(h)
        h = self.resnet("mid_block.resnets.0", h, temb)
        h = self.transformer("mid_block.attentions.0", h, ctx, self._heads(nlev - 1), self._layers(nlev - 1))
        h = self.resnet("mid_block.resnets.1", h, temb)
        for i, typ in enumerate(cfg["up_block_types"]):
            lvl = nlev - 1 - i
            for j in range(cfg["layers_per_block"] + 1):
                h = torch.cat([h, skips.pop()], dim=1)
                h = self.resnet(f"up_blocks.{i}.resnets.{j}", h, temb)
                if typ == "CrossAttnUpBlock2D":
                    h = self.transformer(f"up_blocks.{i}.attentions.{j}", h, ctx, self._heads(lvl), self._layers(lvl))
            if i < nlev - 1:
                h = F.interpolate(h, scale_factor=2.0, mode="nearest")
                h = self.conv(f"up_blocks.{i}.upsamplers.0.conv", h)
        h = F.silu(self.gn("conv_norm_out", h, cfg["norm_num_groups"], cfg["norm_eps"]))
        return self.conv("conv_out", h)


# ------------------------------------------------------------------ scheduler / loop
def ddim_step(eps_cfg_in, t_idx, latents, a_t, a_p, guidance):
    """CFG combine + DDIMScheduler.step (eta 0) in diffusers' op order (fp16 tensors, fp32
    0-d scheduler scalars)."""
    u, c = eps_cfg_in.chunk(2)
    eps = u + guidance * (c - u)
    at = a_t[t_idx]
    ap = a_p[t_idx]
    bt = 1 - at
    x0 = (latents - bt ** 0.5 * eps) / at ** 0.5
    direction = (1 - ap) ** 0.5 * eps
    return ap ** 0.5 * x0 + direction


def ddim_tables(num_inference_steps, num_train=1000, beta_start=0.00085, beta_end=0.012, steps_offset=1):
    """DDIMScheduler.set_timesteps ("leading", scaled_linear betas, set_alpha_to_one False):
    (timesteps int64 [S], alpha_t f32 [S], alpha_prev f32 [S])."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train, dtype=torch.float32) ** 2
    ac = torch.cumprod(1.0 - betas, dim=0)
    ratio = num_train // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64) + steps_offset
    a_t = torch.stack([ac[int(t)] for t in ts])
    a_p = torch.stack([ac[int(t) - ratio] if int(t) - ratio >= 0 else ac[0] for t in ts])
    return torch.from_numpy(ts), a_t, a_p


@torch.no_grad()
def denoise(unet, latents, ctx, timesteps, a_t, a_p, guidance=7.5, steps=None):
    """The reference's pipeline loop on CPU: returns latents after `steps` steps."""
    lat = latents.to(F16)
    n = len(timesteps) if steps is None else steps
    for i in range(n):
        x = torch.cat([lat] * 2)
        eps = unet.forward(x, int(timesteps[i]), ctx)
        lat = ddim_step(eps, i, lat, a_t, a_p, guidance)
    return lat


# ------------------------------------------------------------------ Euler discrete (SDXL)
def euler_tables(num_inference_steps, num_train=1000, beta_start=0.00085, beta_end=0.012, steps_offset=1):
    """EulerDiscreteScheduler.set_timesteps ("leading", linear interpolation): (timesteps f32,
    sigmas f32 [S + 1], init_noise_sigma 0-d f32)."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train, dtype=torch.float32) ** 2
    ac = torch.cumprod(1.0 - betas, dim=0)
    ratio = num_train // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.float32) + steps_offset
    sig = (((1 - ac) / ac) ** 0.5).numpy()
    sig = np.interp(ts, np.arange(0, len(sig)), sig)
    sigmas = torch.from_numpy(np.concatenate([sig, [0.0]]).astype(np.float32))
    return torch.from_numpy(ts), sigmas, (sigmas.max() ** 2 + 1) ** 0.5


def euler_step(eps_cfg_in, i, latents, sigmas, guidance):
    """CFG + EulerDiscreteScheduler.step (epsilon, s_churn 0) in diffusers' op order."""
    u, c = eps_cfg_in.chunk(2)
    eps = u + guidance * (c - u)
    sample = latents.to(torch.float32)
    sigma_hat = sigmas[i] * (0.0 + 1)
    pred = sample - sigma_hat * eps
    deriv = (sample - pred) / sigma_hat
    dt = sigmas[i + 1] - sigma_hat
    return (sample + deriv * dt).to(eps.dtype)


@torch.no_grad()
def denoise_euler(unet, latents, ctx, add_emb, timesteps, sigmas, init_sigma, guidance=5.0, steps=None):
    """The SDXL pipeline loop on CPU: latents * init_noise_sigma, then per step
    scale_model_input (/ (sigma ** 2 + 1) ** 0.5), UNet, CFG, Euler step."""
    lat = latents.to(F16) * init_sigma
    n = len(timesteps) if steps is None else steps
    for i in range(n):
        x = torch.cat([lat] * 2)
        x = x / ((sigmas[i] ** 2 + 1) ** 0.5)
        eps = unet.forward(x, float(timesteps[i]), ctx, add_emb)
        lat = euler_step(eps, i, lat, sigmas, guidance)
    return lat


# ------------------------------------------------------------------ PNDM (SD1.5's scheduler_config)
def pndm_tables(num_inference_steps, num_train=1000, beta_start=0.00085, beta_end=0.012, steps_offset=1):
    """PNDMScheduler.set_timesteps with skip_prk_steps: the PLMS timesteps (second one repeated)."""
    ratio = num_train // num_inference_steps
    t = (np.arange(0, num_inference_steps) * ratio).round().astype(np.int64) + steps_offset
    return np.concatenate([t[:-1], t[-2:-1], t[-1:]])[::-1].copy(), ratio


class PNDMRef:
    """PNDMScheduler.step_plms restated with torch-CPU ops in diffusers' order (fp16 sample /
    model_output tensors, fp32 0-d alphas): the multistep history ets, the counter-1 restart."""

    def __init__(self, num_train=1000, beta_start=0.00085, beta_end=0.012, num_inference_steps=50):
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train, dtype=torch.float32) ** 2
        self.ac = torch.cumprod(1.0 - betas, dim=0)
        self.final = self.ac[0]
        self.ratio = num_train // num_inference_steps
        self.ets, self.counter, self.cur = [], 0, None

    def _prev_sample(self, sample, t, prev_t, mo):
        a_t = self.ac[t]
        a_p = self.ac[prev_t] if prev_t >= 0 else self.final
        b_t, b_p = 1 - a_t, 1 - a_p
        sample_coeff = (a_p / a_t) ** 0.5
        denom = a_t * b_p ** 0.5 + (a_t * b_t * a_p) ** 0.5
        return sample_coeff * sample - (a_p - a_t) * mo / denom

    def step(self, mo, t, sample):
        prev_t = t - self.ratio
        if self.counter != 1:
            self.ets = self.ets[-3:]
            self.ets.append(mo)
        else:
            prev_t = t
            t = t + self.ratio
        if len(self.ets) == 1 and self.counter == 0:
            self.cur = sample
        elif len(self.ets) == 1 and self.counter == 1:
            mo = (mo + self.ets[-1]) / 2
            sample = self.cur
            self.cur = None
        elif len(self.ets) == 2:
            mo = (3 * self.ets[-1] - self.ets[-2]) / 2
        elif len(self.ets) == 3:
            mo = (23 * self.ets[-1] - 16 * self.ets[-2] + 5 * self.ets[-3]) / 12
        else:
            mo = (1 / 24) * (55 * self.ets[-1] - 59 * self.ets[-2] + 37 * self.ets[-3] - 9 * self.ets[-4])
        prev = self._prev_sample(sample, t, prev_t, mo)
        self.counter += 1
        return prev


@torch.no_grad()
def denoise_pndm(unet, latents, ctx, num_inference_steps, guidance=7.5, steps=None):
    """The SD pipeline loop with PNDMScheduler (skip_prk_steps) on CPU."""
    ts, _ = pndm_tables(num_inference_steps)
    sch = PNDMRef(num_inference_steps=num_inference_steps)
    lat = latents.to(F16)
    n = len(ts) if steps is None else steps
    for i in range(n):
        eps = unet.forward(torch.cat([lat] * 2), int(ts[i]), ctx)
        u, c = eps.chunk(2)
        lat = sch.step(u + guidance * (c - u), int(ts[i]), lat)
    return lat
