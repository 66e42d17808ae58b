"""CPU restatement of diffusers' AutoencoderKL decode path - TEST INFRASTRUCTURE ONLY (tests/ and
tests/golden/ scripts; the product never imports oracle/).

diffusers is not installed here (parity of the architecture itself is unpinned, as for the UNet:
DESIGN.md §4); the restatement follows diffusers' Decoder / UNetMidBlock2D / UpDecoderBlock2D /
ResnetBlock2D (temb None, eps 1e-6, output_scale_factor 1) / Attention + AttnProcessor2_0
(group_norm, heads 1, residual_connection, rescale 1) / Upsample2D (nearest 2x + conv) and the
pipelines' ``vae.decode(latents / scaling_factor [+ shift])`` + VaeImageProcessor.postprocess,
op for op in torch-CPU fp16 ("half") or with every GEMM / conv / norm / attention in fp32 rounded
once ("fp32").  Fake-quant of the decoder (the reference's quantVAE swaps decoder layers only,
models/StableDiffusion1_x.py:58-67) reuses RefUNet's golden-pinned layer ops.
"""
import torch
import torch.nn.functional as F

from .unet_ref import RefUNet, quantize_state_dict

F16 = torch.float16


class RefVAEDecoder(RefUNet):
    """cfg: dict of VAEConfig fields; sd: {key: tensor} (decoder.* and post_quant_conv.*)."""

    def __init__(self, cfg, sd, qc=None, variant="half"):
        dec = {k: v for k, v in sd.items() if k.startswith("decoder.")}
        rest = {k: v for k, v in sd.items() if not k.startswith("decoder.")}
        RefUNet.__init__(self, cfg, dec, qc, variant)
        self.sd.update({k: v.detach().to("cpu", F16).contiguous() for k, v in rest.items()})
        self.eps = 1e-6

    def resnet(self, p, x):
        g = self.cfg["norm_num_groups"]
        h = F.silu(self.gn(p + ".norm1", x, g, self.eps))
        h = self.conv(p + ".conv1", h)
        h = F.silu(self.gn(p + ".norm2", h, g, self.eps))
        h = self.conv(p + ".conv2", h)
        if p + ".conv_shortcut.weight" in self.sd:
            x = self.conv(p + ".conv_shortcut", x)
        return (x + h) / 1.0

    def attn(self, p, x):
        b, c, hh, ww = x.shape
        res = x
        h = x.view(b, c, hh * ww).transpose(1, 2)
        h = self.gn(p + ".group_norm", h.transpose(1, 2), self.cfg["norm_num_groups"], self.eps).transpose(1, 2)
        q = self.lin(p + ".to_q", h).view(b, -1, 1, c).transpose(1, 2)
        k = self.lin(p + ".to_k", h).view(b, -1, 1, c).transpose(1, 2)
        v = self.lin(p + ".to_v", h).view(b, -1, 1, c).transpose(1, 2)
        o = self.ops.scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False)
        o = o.transpose(1, 2).reshape(b, -1, c).to(q.dtype)
        o = self.lin(p + ".to_out.0", o)
        o = o.transpose(-1, -2).reshape(b, c, hh, ww)
        return (o + res) / 1.0

    @torch.no_grad()
    def decode(self, latents):
        """Denoised latents [N, latent_channels, h, w] fp16 -> decoder output [N, 3, 8h, 8w] fp16."""
        cfg = self.cfg
        z = latents.to(F16) / cfg["scaling_factor"]
        if cfg.get("shift_factor") is not None:
            z = z + cfg["shift_factor"]
        if cfg.get("use_post_quant_conv", True):
            z = self.conv("post_quant_conv", z)
        h = self.conv("decoder.conv_in", z)
        h = self.resnet("decoder.mid_block.resnets.0", h)
        if cfg.get("mid_block_add_attention", True):
            h = self.attn("decoder.mid_block.attentions.0", h)
        h = self.resnet("decoder.mid_block.resnets.1", h)
        nlev = len(cfg["block_out_channels"])
        for i in range(nlev):
            for j in range(cfg["layers_per_block"] + 1):
                h = self.resnet(f"decoder.up_blocks.{i}.resnets.{j}", h)
            if i < nlev - 1:
                h = F.interpolate(h, scale_factor=2.0, mode="nearest")
                h = self.conv(f"decoder.up_blocks.{i}.upsamplers.0.conv", h)
        h = F.silu(self.gn("decoder.conv_norm_out", h, cfg["norm_num_groups"], self.eps))
        return self.conv("decoder.conv_out", h)


def postprocess(img):
    """VaeImageProcessor.postprocess denormalize: (image / 2 + 0.5).clamp(0, 1) (Half ops)."""
    return (img / 2 + 0.5).clamp(0, 1)


def to_uint8(img):
    """numpy_to_pil's (images * 255).round().astype("uint8") on the float32 NHWC image."""
    a = img.permute(0, 2, 3, 1).float().numpy()
    return (a * 255).round().astype("uint8")


__all__ = ["RefVAEDecoder", "postprocess", "to_uint8", "quantize_state_dict"]
