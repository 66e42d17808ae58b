"""Host-side checks of the text encoder / VAE components (no GPU): checkpoint key layout against
transformers, tokenizer framing and pooled-row rule, the VAE oracle's shapes, lazy pipeline
components and their save / reload through a local diffusers directory."""
import json

import pytest
import torch


def test_clip_keys_match_transformers():
    from transformers import CLIPTextConfig as HC
    from transformers import CLIPTextModelWithProjection as HP
    from qdiff.clip import CLIPTextModel, tiny_clip_config
    for proj in (None, 32):
        cfg = tiny_clip_config(projection_dim=proj)
        ours = set(CLIPTextModel(cfg).state_dict())
        if proj:
            theirs = set(HP(HC(**cfg.to_transformers())).state_dict())
        else:
            from transformers import CLIPTextModel as HM
            theirs = {"text_model." + k for k in HM(HC(**cfg.to_transformers())).state_dict()}
        theirs = {k for k in theirs if "position_ids" not in k}
        assert ours == theirs, ours ^ theirs


def test_tokenizer_framing_and_eos_rule():
    from qdiff.clip import BOS, EOS, HashTokenizer, eos_positions
    tok = HashTokenizer()
    ids = tok(["a red cube", "", "word " * 200])
    assert ids.shape == (3, 77) and ids.dtype == torch.int64
    assert (ids[:, 0] == BOS).all()
    assert ids[0, 4] == EOS and (ids[0, 5:] == EOS).all() and (ids[0, 1:4] < BOS).all()
    assert ids[1, 1] == EOS and ids[2, 76] == EOS
    assert eos_positions(ids, 2).tolist() == [4, 1, 76]           # argmax rule (legacy configs)
    assert eos_positions(ids, EOS).tolist() == [4, 1, 76]         # first EOS
    tok2 = HashTokenizer(pad_id=0)
    ids2 = tok2(["a red cube"])
    assert ids2[0, 4] == EOS and (ids2[0, 5:] == 0).all()


def test_vae_oracle_shapes_and_postprocess():
    import dataclasses
    from oracle.vae_ref import RefVAEDecoder, postprocess, to_uint8
    from qdiff.vae import AutoencoderKL, tiny_vae_config
    for lc in (4, 16):
        cfg = tiny_vae_config(lc)
        vae = AutoencoderKL(cfg).half().init_synthetic(1)
        cd = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(cfg).items()}
        lat = torch.randn(1, lc, 8, 8).half()
        y = RefVAEDecoder(cd, vae.state_dict(), None, variant="fp32").decode(lat)
        assert y.shape == (1, 3, 64, 64)
        img = postprocess(y)
        assert float(img.min()) >= 0 and float(img.max()) <= 1
        assert to_uint8(img).shape == (1, 64, 64, 3)


def test_lazy_components_save_and_reload(tmp_path):
    from qdiff.clip import CLIPTextModel
    from qdiff.pipeline_io import load_pipeline
    from qdiff.vae import AutoencoderKL
    p = load_pipeline("synthetic:tiny", device="cpu", seed=2)
    assert p.component_names() == ["unet", "text_encoder", "vae"]
    assert "text_encoder" not in p.__dict__ and "vae" not in p.__dict__     # not built yet
    te, vae = p.text_encoder, p.vae
    assert isinstance(te, CLIPTextModel) and isinstance(vae, AutoencoderKL)
    assert te.config.hidden_size == p.unet.config.cross_attention_dim
    p.save_pretrained(str(tmp_path))
    idx = json.load(open(tmp_path / "model_index.json"))
    assert idx["text_encoder"] == ["transformers", "CLIPTextModel"] and idx["vae"] == ["diffusers", "AutoencoderKL"]
    q = load_pipeline(str(tmp_path), device="cpu")
    assert q.component_names() == ["unet", "text_encoder", "vae"]
    for a, b in ((te, q.text_encoder), (vae, q.vae)):
        sa, sb = a.state_dict(), b.state_dict()
        assert set(sa) == set(sb) and all(torch.equal(sa[k], sb[k]) for k in sa)
    assert q.text_encoder.config == te.config and q.vae.config == vae.config


def test_vae_legacy_attention_names():
    from qdiff.pipeline_io import _clip_keys, _vae_keys
    assert _vae_keys("decoder.mid_block.attentions.0.query.weight") == "decoder.mid_block.attentions.0.to_q.weight"
    assert _vae_keys("decoder.mid_block.attentions.0.proj_attn.bias") == "decoder.mid_block.attentions.0.to_out.0.bias"
    assert _clip_keys("encoder.layers.0.mlp.fc1.weight") == "text_model.encoder.layers.0.mlp.fc1.weight"
    assert _clip_keys("text_projection.weight") == "text_projection.weight"


def test_sdxl_and_sd3_synthetic_encoder_widths():
    from qdiff.pipeline_io import load_pipeline
    p = load_pipeline("synthetic:sdxl-tiny", device="cpu")
    u = p.unet.config
    assert p.text_encoder.config.hidden_size + p.text_encoder_2.config.hidden_size == u.cross_attention_dim
    assert p.text_encoder_2.config.projection_dim == u.projection_class_embeddings_input_dim - 6 * u.addition_time_embed_dim
    p = load_pipeline("synthetic:sd35-tiny", device="cpu")
    t = p.transformer.config
    assert p.text_encoder.config.projection_dim + p.text_encoder_2.config.projection_dim == t.pooled_projection_dim
    assert p.vae.config.latent_channels == t.in_channels == 16
    with pytest.raises(AttributeError):
        p.tokenizer_3
