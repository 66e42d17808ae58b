"""qdiff: MI355X-native quantized-diffusion denoising path (drop-in for the diffusion adapters
of maani3/Quantization---Diffusion-Models).  Import as ``qdiff`` via ``qdiff_boot``."""
from .config import AwqConfig
from .fake_quant import (WxAxConv2d, WxAxLinear, quantize_activation_per_channel_absmax,
                         quantize_activation_per_channel_group_absmax, quantize_activation_per_tensor_absmax,
                         quantize_activation_per_token_absmax, quantize_weight_absmax,
                         quantize_weight_per_channel_absmax, quantize_weight_per_tensor_absmax)
from .models import AWQ, StableDiffusion1_x, StableDiffusion3_5, StableDiffusionXL
from .quantizer import AwqQuantizer, SqQuantizer
from .unet import SD15, SDXL, UNet2DConditionModel, UNetConfig, tiny_config

__all__ = [
    "AWQ", "AwqConfig", "AwqQuantizer", "SqQuantizer", "StableDiffusion1_x", "StableDiffusionXL",
    "StableDiffusion3_5", "UNet2DConditionModel", "UNetConfig", "SD15", "SDXL", "tiny_config",
    "WxAxLinear", "WxAxConv2d", "quantize_weight_absmax", "quantize_weight_per_channel_absmax",
    "quantize_weight_per_tensor_absmax", "quantize_activation_per_token_absmax",
    "quantize_activation_per_channel_absmax", "quantize_activation_per_channel_group_absmax",
    "quantize_activation_per_tensor_absmax",
]
