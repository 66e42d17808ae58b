"""CLIP text encoder (transformers CLIPTextModel / CLIPTextModelWithProjection) on the fused HIP
path, and the pipelines' prompt encoding (diffusers StableDiffusionPipeline /
StableDiffusionXLPipeline / StableDiffusion3Pipeline ``encode_prompt``).

The reference runs the checkpoint's text encoder(s) inside ``self.pipeline(prompt=...)``
(models/base.py:848) and can fake-quantize them (``quantTextEncoder``: the swap walks
``pipeline.text_encoder.named_children()``, models/StableDiffusion1_x.py:49-56; the per-token
output quant of ``q_proj`` / ``k_proj`` / ``v_proj`` follows quantize/quantizer.py's child-name
rule).  Module and parameter names are the transformers ones (``text_model.encoder.layers.N.
self_attn.q_proj`` ...), so checkpoints load unchanged.

One encoder layer on device: LayerNorm -> q|k|v as one GEMM (bias in the epilogue) -> causal
attention (qd_attention_causal) -> out_proj + residual (epilogue) -> LayerNorm -> fc1 ->
quick_gelu / gelu -> fc2 + residual (epilogue).
"""
import zlib
from dataclasses import dataclass, fields
from typing import Optional

import torch
from torch import nn

from . import kernels as K
from .fake_quant import WxAxLinear
from .mmdit import _stacked_operand
from .unet import _f16, run_linear

BOS, EOS = 49406, 49407


@dataclass(frozen=True)
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    hidden_act: str = "quick_gelu"
    layer_norm_eps: float = 1e-5
    projection_dim: Optional[int] = None   # CLIPTextModelWithProjection: text_projection width
    eos_token_id: int = 2                  # 2 (SD1.5's config): pooled row = argmax(ids)
    pad_token_id: int = 1

    @classmethod
    def from_transformers(cls, d: dict, with_projection=False):
        names = {f.name for f in fields(cls)}
        kw = {k: v for k, v in d.items() if k in names}
        if not with_projection:
            kw["projection_dim"] = None
        return cls(**kw)

    def to_transformers(self):
        d = {f.name: getattr(self, f.name) for f in fields(self)}
        if d["projection_dim"] is None:
            d.pop("projection_dim")
        return d


CLIP_L = CLIPTextConfig()                                      # SD1.5 text_encoder (ViT-L/14)
CLIP_L_PROJ = CLIPTextConfig(projection_dim=768, eos_token_id=EOS)       # SDXL / SD3 text_encoder
CLIP_G = CLIPTextConfig(hidden_size=1280, intermediate_size=5120, num_hidden_layers=32, num_attention_heads=20,
                        hidden_act="gelu", projection_dim=1280, eos_token_id=EOS, pad_token_id=0)  # OpenCLIP bigG


def tiny_clip_config(hidden=64, heads=2, layers=2, projection_dim=None, act="quick_gelu"):
    return CLIPTextConfig(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=layers,
                          num_attention_heads=heads, hidden_act=act, projection_dim=projection_dim,
                          eos_token_id=2 if projection_dim is None else EOS)


# ------------------------------------------------------------------ module tree (transformers names)
class _Embeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.token_embedding = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size)


class _Attention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        c = cfg.hidden_size
        self.heads = cfg.num_attention_heads
        self.k_proj = nn.Linear(c, c)
        self.v_proj = nn.Linear(c, c)
        self.q_proj = nn.Linear(c, c)
        self.out_proj = nn.Linear(c, c)


class _MLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.fc1 = nn.Linear(cfg.hidden_size, cfg.intermediate_size)
        self.fc2 = nn.Linear(cfg.intermediate_size, cfg.hidden_size)


class _Layer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.self_attn = _Attention(cfg)
        self.layer_norm1 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.mlp = _MLP(cfg)
        self.layer_norm2 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.hidden_act = cfg.hidden_act


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layers = nn.ModuleList([_Layer(cfg) for _ in range(cfg.num_hidden_layers)])


class _TextTransformer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.final_layer_norm = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)


class CLIPTextModel(nn.Module):
    """CLIPTextModel (projection_dim None) or CLIPTextModelWithProjection."""

    def __init__(self, cfg: CLIPTextConfig = CLIP_L):
        super().__init__()
        self.config = cfg
        self.text_model = _TextTransformer(cfg)
        self.text_projection = (nn.Linear(cfg.hidden_size, cfg.projection_dim, bias=False)
                                if cfg.projection_dim else None)

    @torch.no_grad()
    def init_synthetic(self, seed=0):
        """Embeddings N(0, 0.02^2) (transformers' init), linears N(0, 1/fan_in), biases 0,
        LayerNorm gamma 1 / beta 0; CPU generator (device independent)."""
        gen = torch.Generator("cpu").manual_seed(seed)
        for name, p in self.named_parameters():
            if "embedding" in name:
                p.copy_((torch.randn(p.shape, generator=gen) * 0.02).to(p.dtype))
            elif name.endswith("weight") and p.dim() >= 2:
                p.copy_((torch.randn(p.shape, generator=gen) / p.shape[1] ** 0.5).to(p.dtype))
            elif name.endswith("bias"):
                p.zero_()
            else:
                p.fill_(1.0)
        return self

    def forward(self, *a, **k):  # pragma: no cover - the pipelines call encode()
        raise RuntimeError("use CLIPTextModel.encode(input_ids) (fused HIP path)")

    @torch.no_grad()
    def encode(self, input_ids, hidden_state=-1, pooled=False):
        """input_ids int64 [B, S] -> (hidden [B, S, C], pooled or None).
        hidden_state -1: last_hidden_state (final LayerNorm applied), -2: hidden_states[-2] (the
        input of the last layer, no final norm; SDXL / SD3 without clip_skip).  pooled: the EOS
        row of the final-normed last state (the text_projection applied when present)."""
        cfg = self.config
        tm = self.text_model
        ids = input_ids.to(self.text_model.final_layer_norm.weight.device, torch.int64).contiguous()
        b, s = ids.shape
        h = K.embed_tokens(ids, _f16(tm.embeddings.token_embedding.weight), _f16(tm.embeddings.position_embedding.weight))
        layers = tm.encoder.layers
        nrun = len(layers) if (hidden_state == -1 or pooled) else len(layers) + 1 + hidden_state
        out = h if nrun == 0 else None
        for i in range(nrun):
            h = _layer_fwd(layers[i], h, b, s)
            if hidden_state != -1 and i == len(layers) + hidden_state:
                out = h
        pool = None
        if hidden_state == -1 or pooled:
            ln = tm.final_layer_norm
            last = K.layernorm(h, ln.eps, _f16(ln.weight), _f16(ln.bias))
            if hidden_state == -1:
                out = last
            if pooled:
                idx = torch.arange(b, dtype=torch.int64) * s + eos_positions(input_ids.cpu(), cfg.eos_token_id)
                pool = K.gather_rows(last, idx.to(h.device))
                if self.text_projection is not None:
                    pool = run_linear(self.text_projection, pool)
        return out.view(b, s, -1), pool


def eos_positions(ids, eos_token_id):
    """transformers CLIPTextModel's pooled row: argmax(ids) when eos_token_id == 2 (the legacy
    configs), else the first occurrence of eos_token_id."""
    if eos_token_id == 2:
        return ids.to(torch.int32).argmax(dim=-1).to(torch.int64)
    return (ids.to(torch.int32) == eos_token_id).int().argmax(dim=-1).to(torch.int64)


def _layer_fwd(layer, h, b, s):
    """CLIPEncoderLayer.forward on token-major h [B*S, C]."""
    at = layer.self_attn
    c = h.shape[1]
    ln1 = layer.layer_norm1
    x = K.layernorm(h, ln1.eps, _f16(ln1.weight), _f16(ln1.bias))
    op = _stacked_operand(at, "_qd_qkv", [at.q_proj, at.k_proj, at.v_proj], allow_out_quant=True)
    if op is not None:
        w, fmt, scl, g, bias, wf, _ = op
        J = K.linear(x, w, fmt, scl, g, bias=bias, weight_f16=wf)
        oq = at.q_proj.output_quant_name if isinstance(at.q_proj, WxAxLinear) else "None"
        if oq != "None":  # per-token output fake-quant of each projection over its own C columns
            y2 = J.view(-1, c)
            K.act_fakequant(y2, oq, at.q_proj.n_bits_A, out=y2)
        J = J.view(b, s, 3 * c)
        q, k, v = J[:, :, :c], J[:, :, c:2 * c], J[:, :, 2 * c:]
    else:
        q, k, v = (run_linear(l, x).view(b, s, c) for l in (at.q_proj, at.k_proj, at.v_proj))
    o = K.attention_causal(q, k, v, at.heads)
    h = run_linear(at.out_proj, o.view(b * s, c), residual=h)
    ln2 = layer.layer_norm2
    x = K.layernorm(h, ln2.eps, _f16(ln2.weight), _f16(ln2.bias))
    f = run_linear(layer.mlp.fc1, x)
    f = K.clip_act(f, layer.hidden_act, out=f)
    return run_linear(layer.mlp.fc2, f, residual=h)


# ------------------------------------------------------------------ tokenizers
class HashTokenizer:
    """Deterministic stand-in for the CLIP BPE tokenizer of synthetic checkpoints (no vocab files
    exist offline): lower-cased whitespace words -> ids in [0, 49405) by crc32; BOS / EOS framing,
    truncation to max_length - 1 + EOS, padding with `pad_id` (EOS for SD1.5, 0 for bigG)."""

    def __init__(self, model_max_length=77, pad_id=EOS, vocab_size=49408):
        self.model_max_length = model_max_length
        self.pad_id = pad_id
        self.vocab_size = vocab_size

    def __call__(self, prompts, max_length=None):
        n = max_length or self.model_max_length
        out = torch.full((len(prompts), n), self.pad_id, dtype=torch.int64)
        for i, p in enumerate(prompts):
            toks = [zlib.crc32(w.encode()) % min(BOS, self.vocab_size - 2) for w in p.lower().split()]
            seq = [BOS] + toks[: n - 2] + [EOS]
            out[i, : len(seq)] = torch.tensor(seq)
        return out


class HFTokenizer:
    """A checkpoint's own tokenizer/ (vocab.json + merges.txt) through transformers' CLIPTokenizer
    (host-side; padding="max_length", truncation=True, as the pipelines call it)."""

    def __init__(self, path):
        from transformers import CLIPTokenizer
        self.tok = CLIPTokenizer.from_pretrained(path, local_files_only=True)
        self.model_max_length = self.tok.model_max_length

    def __call__(self, prompts, max_length=None):
        r = self.tok(list(prompts), padding="max_length", max_length=max_length or self.model_max_length,
                     truncation=True, return_tensors="pt")
        return r.input_ids.to(torch.int64)


def load_tokenizer(path, pad_id=EOS):
    import os
    if path and os.path.exists(os.path.join(path, "vocab.json")) and os.path.exists(os.path.join(path, "merges.txt")):
        return HFTokenizer(path)
    return HashTokenizer(pad_id=pad_id)


# ------------------------------------------------------------------ pipelines' encode_prompt
def _as_list(p, n=None):
    if p is None:
        return None
    out = [p] if isinstance(p, str) else list(p)
    if n is not None and len(out) == 1 and n > 1:
        out = out * n
    return out


@torch.no_grad()
def encode_sd15(pipe, prompt, negative_prompt=None):
    """StableDiffusionPipeline.encode_prompt (clip_skip None, no attention mask): [2B, 77, C]
    = cat(negative (default ""), positive) last_hidden_state."""
    te, tok = pipe.text_encoder, pipe.tokenizer
    prompts = _as_list(prompt)
    negs = _as_list(negative_prompt if negative_prompt is not None else "", len(prompts))
    pe, _ = te.encode(tok(prompts))
    ne, _ = te.encode(tok(negs, max_length=pe.shape[1]))
    return torch.cat([ne, pe]).contiguous()


@torch.no_grad()
def _sdxl_pair(pipe, prompts):
    e1, _ = pipe.text_encoder.encode(pipe.tokenizer(prompts), hidden_state=-2)
    e2, pooled = pipe.text_encoder_2.encode(pipe.tokenizer_2(prompts), hidden_state=-2, pooled=True)
    return K.concat_c(e1.contiguous(), e2.contiguous()), pooled


@torch.no_grad()
def encode_sdxl(pipe, prompt, negative_prompt=None, force_zeros_for_empty_prompt=True):
    """StableDiffusionXLPipeline.encode_prompt: both encoders' hidden_states[-2] concatenated
    along features, pooled = text_encoder_2's text_embeds; negative embeddings are zeros when no
    negative prompt is given (force_zeros_for_empty_prompt).  Returns (ctx [2B, 77, C1 + C2],
    pooled [2B, P]) negative first."""
    prompts = _as_list(prompt)
    pe, pp = _sdxl_pair(pipe, prompts)
    if negative_prompt is None and force_zeros_for_empty_prompt:
        ne, npool = torch.zeros_like(pe), torch.zeros_like(pp)
    else:
        ne, npool = _sdxl_pair(pipe, _as_list(negative_prompt if negative_prompt is not None else "", len(prompts)))
    return torch.cat([ne, pe]).contiguous(), torch.cat([npool, pp]).contiguous()


@torch.no_grad()
def _sd3_one(pipe, prompts, joint_dim):
    el, pl = pipe.text_encoder.encode(pipe.tokenizer(prompts), hidden_state=-2, pooled=True)
    eg, pg = pipe.text_encoder_2.encode(pipe.tokenizer_2(prompts), hidden_state=-2, pooled=True)
    clip = K.concat_c(el.contiguous(), eg.contiguous())                    # [B, 77, Cl + Cg]
    b, s, cc = clip.shape
    out = torch.zeros(b, 2 * s, joint_dim, dtype=torch.float16, device=clip.device)
    out[:, :s, :cc] = clip      # clip embeds padded to joint_attention_dim; T5 part (no text_encoder_3): zeros
    return out, K.concat_c(pl.contiguous(), pg.contiguous())


@torch.no_grad()
def encode_sd3(pipe, prompt, negative_prompt=None, joint_dim=4096):
    """StableDiffusion3Pipeline.encode_prompt without text_encoder_3 (T5 absent: its embeddings are
    zeros of [B, 77, joint_attention_dim], as diffusers does): prompt_embeds [2B, 154, joint_dim]
    and pooled [2B, Pl + Pg], negative ("" by default) first."""
    prompts = _as_list(prompt)
    pe, pp = _sd3_one(pipe, prompts, joint_dim)
    ne, npool = _sd3_one(pipe, _as_list(negative_prompt if negative_prompt is not None else "", len(prompts)),
                         joint_dim)
    return torch.cat([ne, pe]).contiguous(), torch.cat([npool, pp]).contiguous()
