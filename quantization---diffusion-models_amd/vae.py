"""AutoencoderKL decoder (diffusers) on the fused NHWC HIP path: latents -> images.

The reference's pipelines decode with ``vae.decode(latents / scaling_factor)`` whenever
``output_type != "latent"`` (models/base.py:848 passes output_type through; ``None`` gives
VaeImageProcessor's "np" images), and ``quantVAE`` fake-quantizes the DECODER only (the swap walks
``pipeline.vae.decoder.named_children()``, models/StableDiffusion1_x.py:58-67).  Parameter names
are diffusers' (``decoder.up_blocks.N.resnets.M.conv1`` ...); the encoder half of the checkpoint
is never used by text-to-image pipelines and is not built.

Device path, NHWC fp16 end to end: prescale (qd_vae_prescale) -> post_quant_conv -> conv_in ->
mid block (resnet, single-head 512-wide self-attention, resnet) -> up blocks (resnets, conv with
the nearest 2x upsample fused into its im2col addressing) -> GroupNorm+SiLU -> conv_out ->
postprocess (qd_vae_postprocess: denormalize, clamp, fp16 NCHW and/or uint8).  Resnet blocks
use the UNet's kernels (GroupNorm+SiLU with the consumer conv's input fake-quant fused, conv
output fake-quant applied inside the next GroupNorm).
"""
from dataclasses import dataclass, fields
from typing import Optional, Tuple

import torch
from torch import nn

from . import kernels as K
from .mmdit import _stacked_operand
from .unet import _f16, conv_qbits, run_conv, run_linear


@dataclass(frozen=True)
class VAEConfig:
    in_channels: int = 3
    out_channels: int = 3
    latent_channels: int = 4
    block_out_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    scaling_factor: float = 0.18215
    shift_factor: Optional[float] = None
    use_post_quant_conv: bool = True
    mid_block_add_attention: bool = True
    sample_size: int = 512
    force_upcast: bool = True

    @classmethod
    def from_diffusers(cls, d: dict):
        names = {f.name for f in fields(cls)}
        kw = {k: v for k, v in d.items() if k in names and v is not None}
        if "block_out_channels" in kw:
            kw["block_out_channels"] = tuple(kw["block_out_channels"])
        if d.get("shift_factor") is None:
            kw["shift_factor"] = None
        return cls(**kw)

    def to_diffusers(self):
        d = {f.name: getattr(self, f.name) for f in fields(self)}
        d["block_out_channels"] = list(d["block_out_channels"])
        d["_class_name"] = "AutoencoderKL"
        return d


SD_VAE = VAEConfig()                                                      # SD1.x
SDXL_VAE = VAEConfig(scaling_factor=0.13025, sample_size=1024)
SD3_VAE = VAEConfig(latent_channels=16, scaling_factor=1.5305, shift_factor=0.0609, use_post_quant_conv=False,
                    sample_size=1024)


def tiny_vae_config(latent_channels=4, **kw):
    """Four levels like the real decoder (8x upsampling), narrow and one resnet deep per level."""
    base = dict(latent_channels=latent_channels, block_out_channels=(16, 32, 32, 32), layers_per_block=1,
                norm_num_groups=8, sample_size=128)
    if latent_channels == 16:
        base.update(scaling_factor=1.5305, shift_factor=0.0609, use_post_quant_conv=False)
    base.update(kw)
    return VAEConfig(**base)


# ------------------------------------------------------------------ module tree (diffusers names)
class VAEResnetBlock(nn.Module):
    def __init__(self, cin, cout, groups, eps=1e-6):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.norm2 = nn.GroupNorm(groups, cout, eps=eps, affine=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None


class VAEAttention(nn.Module):
    """diffusers Attention(heads=1, dim_head=C, norm_num_groups, residual_connection=True, bias=True)."""

    def __init__(self, ch, groups):
        super().__init__()
        self.heads = 1
        self.group_norm = nn.GroupNorm(groups, ch, eps=1e-6, affine=True)
        self.to_q = nn.Linear(ch, ch)
        self.to_k = nn.Linear(ch, ch)
        self.to_v = nn.Linear(ch, ch)
        self.to_out = nn.ModuleList([nn.Linear(ch, ch), nn.Dropout(0.0)])


class _Upsample(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, padding=1)


class _MidBlock(nn.Module):
    def __init__(self, ch, groups, attention=True):
        super().__init__()
        self.attentions = nn.ModuleList([VAEAttention(ch, groups)]) if attention else None
        self.resnets = nn.ModuleList([VAEResnetBlock(ch, ch, groups), VAEResnetBlock(ch, ch, groups)])


class _UpBlock(nn.Module):
    def __init__(self, cin, cout, n, groups, upsample):
        super().__init__()
        self.resnets = nn.ModuleList([VAEResnetBlock(cin if i == 0 else cout, cout, groups) for i in range(n)])
        self.upsamplers = nn.ModuleList([_Upsample(cout)]) if upsample else None


class Decoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch = list(reversed(cfg.block_out_channels))
        g = cfg.norm_num_groups
        self.conv_in = nn.Conv2d(cfg.latent_channels, ch[0], 3, padding=1)
        self.mid_block = _MidBlock(ch[0], g, cfg.mid_block_add_attention)
        self.up_blocks = nn.ModuleList()
        prev = ch[0]
        for i, c in enumerate(ch):
            self.up_blocks.append(_UpBlock(prev, c, cfg.layers_per_block + 1, g, i < len(ch) - 1))
            prev = c
        self.conv_norm_out = nn.GroupNorm(g, ch[-1], eps=1e-6, affine=True)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(ch[-1], cfg.out_channels, 3, padding=1)


class AutoencoderKL(nn.Module):
    """The decoder half of diffusers' AutoencoderKL (+ post_quant_conv)."""

    def __init__(self, cfg: VAEConfig = SD_VAE):
        super().__init__()
        self.config = cfg
        self.decoder = Decoder(cfg)
        self.post_quant_conv = (nn.Conv2d(cfg.latent_channels, cfg.latent_channels, 1)
                                if cfg.use_post_quant_conv else None)

    @torch.no_grad()
    def init_synthetic(self, seed=0):
        """Weights N(0, 1/fan_in), biases 0, GroupNorm gamma 1 / beta 0 (CPU generator)."""
        gen = torch.Generator("cpu").manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("weight") and p.dim() >= 2:
                p.copy_((torch.randn(p.shape, generator=gen) / p[0].numel() ** 0.5).to(p.dtype))
            elif name.endswith("bias"):
                p.zero_()
            else:
                p.fill_(1.0)
        return self

    def forward(self, *a, **k):  # pragma: no cover
        raise RuntimeError("use AutoencoderKL.decode_nhwc(latents) / decode_images(...) (fused HIP path)")

    # ---------------------------------------------------------------- device decode
    @torch.no_grad()
    def decode_nhwc(self, lat):
        """lat: NHWC fp16 [N, h, w, Cp] denoised latents (latent_channels valid, as the loops hold
        them) -> decoder output NHWC [N, 8h, 8w, 8] (3 channels valid)."""
        cfg = self.config
        cl = cfg.latent_channels
        cp = (cl + 7) // 8 * 8
        z = K.vae_prescale(lat, cl, cfg.scaling_factor, cfg.shift_factor, cout_pad=cp)
        if self.post_quant_conv is not None:
            z = run_conv(self.post_quant_conv, z, c_valid=cl, co_pad=cp)
        dec = self.decoder
        h = run_conv(dec.conv_in, z, c_valid=cl)
        mb = dec.mid_block
        h = resnet_fwd(mb.resnets[0], h)
        if mb.attentions is not None:
            h = attention_fwd(mb.attentions[0], h)
        h = resnet_fwd(mb.resnets[1], h)
        for blk in dec.up_blocks:
            for res in blk.resnets:
                h = resnet_fwd(res, h)
            if blk.upsamplers is not None:
                h = run_conv(blk.upsamplers[0].conv, h, upsample=True)
        q = conv_qbits(dec.conv_out)
        n = dec.conv_norm_out
        h = K.groupnorm_nhwc(h, n.num_groups, n.eps, _f16(n.weight), _f16(n.bias), silu=True, q_bits=max(q, 0))
        return run_conv(dec.conv_out, h, prequant=q > 0, co_pad=8)

    def samples_per_chunk(self, h, w):
        """Samples decoded per launch sequence: the largest activation (the last up block's input
        at full resolution, block_out_channels[1] channels) stays inside the kernels' 2 GiB
        buffer-addressing range."""
        ch = self.config.block_out_channels
        widest = max(ch[1] if len(ch) > 1 else ch[0], ch[0]) * 8 * h * 8 * w * 2
        return max(1, int(1.9 * 2 ** 30 // widest))

    @torch.no_grad()
    def decode_images(self, lat, output_type="np"):
        """Denoised NHWC latents -> VaeImageProcessor.postprocess output: "pt" fp16 NCHW [N, 3, H, W]
        on the device, "np" float32 [N, H, W, 3] (output_type None in the reference), "pil" a
        list of PIL images."""
        n, h, w, _ = lat.shape
        step = self.samples_per_chunk(h, w)
        want_u8 = output_type == "pil"
        pts, u8s = [], []
        for i in range(0, n, step):
            y = self.decode_nhwc(lat[i:i + step].contiguous())
            a, u = K.vae_postprocess(y, self.config.out_channels, want_nchw=not want_u8, want_u8=want_u8)
            pts.append(a)
            u8s.append(u)
        if output_type == "pil":
            from PIL import Image
            arr = torch.cat(u8s).cpu().numpy()
            return [Image.fromarray(a) for a in arr]
        img = torch.cat(pts)
        if output_type == "pt":
            return img
        return img.cpu().permute(0, 2, 3, 1).float().numpy()


def resnet_fwd(res, x):
    """diffusers ResnetBlock2D without a time embedding (temb_channels None), eps 1e-6."""
    q1 = conv_qbits(res.conv1)
    n1, n2 = res.norm1, res.norm2
    h = K.groupnorm_nhwc(x, n1.num_groups, n1.eps, _f16(n1.weight), _f16(n1.bias), silu=True, q_bits=max(q1, 0))
    sc = run_conv(res.conv_shortcut, x) if res.conv_shortcut is not None else x
    h, spec = run_conv(res.conv1, h, prequant=q1 > 0, defer=True)
    q2 = conv_qbits(res.conv2)
    h = K.groupnorm_nhwc(h, n2.num_groups, n2.eps, _f16(n2.weight), _f16(n2.bias), silu=True, q_bits=max(q2, 0),
                         fq_in=spec)
    return run_conv(res.conv2, h, prequant=q2 > 0, residual=sc)


def attention_fwd(at, x):
    """Attention + AttnProcessor2_0 on NHWC x: group_norm -> to_q | to_k | to_v (one GEMM when the
    projections can share it) -> one C-wide head (qd_attention, head_dim up to 512) -> to_out[0]
    + residual (epilogue)."""
    n, hh, ww, c = x.shape
    s = hh * ww
    gn = at.group_norm
    h = K.groupnorm_nhwc(x, gn.num_groups, gn.eps, _f16(gn.weight), _f16(gn.bias)).view(n * s, c)
    op = _stacked_operand(at, "_qd_qkv", [at.to_q, at.to_k, at.to_v])
    if op is not None:
        w, fmt, scl, g, b, wf, _ = op
        J = K.linear(h, w, fmt, scl, g, bias=b, weight_f16=wf).view(n, s, 3 * c)
        q, k, v = J[:, :, :c], J[:, :, c:2 * c], J[:, :, 2 * c:]
    else:
        q, k, v = (run_linear(l, h).view(n, s, c) for l in (at.to_q, at.to_k, at.to_v))
    o = K.attention(q, k, v, at.heads)
    return run_linear(at.to_out[0], o.view(n * s, c), residual=x.view(n * s, c)).view(n, hh, ww, c)
