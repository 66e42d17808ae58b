"""Full-size pixel-space golden (TEST FIXTURE, computed in the build container whose AVX512-FP16
CPU runs the half oracle's torch-CPU Half kernels at speed):

    python tests/golden/make_pixel_golden.py

SD1.5 at 512x512, one prompt, a short DDIM run (4 steps, CFG 7.5), W8A8 RTN fake-quant UNet:
prompt -> CLIP ViT-L/14 (transformers' CLIPTextModel on the synthetic checkpoint's text-encoder
weights, the library the reference's pipeline runs) -> oracle UNet loop (oracle/unet_ref.py,
golden-pinned fake-quant) -> oracle VAE decode (oracle/vae_ref.py) -> VaeImageProcessor
postprocess -> uint8 (numpy_to_pil's round) - base.py:828-850's generate() with output_type 'pil'.
Both oracle variants (torch-CPU "half" and per-op "fp32") are stored with the latents they
decode, the token ids and a fingerprint of every weight, into tests/golden/pixel_golden.npz;
tests/test_gpu_pixel.py compares the GPU's uint8 images with them.
"""
import dataclasses
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import qdiff_boot  # noqa: E402,F401

from oracle import config_cases as CC  # noqa: E402

OUT = os.path.join(HERE, "pixel_golden.npz")
CASE = dict(model="synthetic:sd15", prompt="an astronaut riding a horse on the moon, detailed photograph",
            res=512, steps=4, guidance=7.5, seed=1010,
            qc=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True))


def hf_clip(cfg, sd, dtype):
    from transformers import CLIPTextConfig as HC
    from transformers import CLIPTextModel as HM
    m = HM(HC(**cfg.to_transformers()))
    sd = {k[len("text_model."):] if k.startswith("text_model.") else k: v for k, v in sd.items()}
    missing, _ = m.load_state_dict({k: v.float() for k, v in sd.items()}, strict=False)
    assert not [k for k in missing if "position_ids" not in k], missing
    return m.to(dtype).eval()


def latents(cfg):
    g = torch.Generator().manual_seed(CASE["seed"])
    hw = CASE["res"] // 8
    return torch.randn(1, cfg.in_channels, hw, hw, generator=g).half()


def main():
    from oracle.unet_ref import RefUNet, ddim_tables, denoise
    from oracle.vae_ref import RefVAEDecoder, postprocess, to_uint8
    from qdiff.pipeline_io import load_pipeline
    torch.set_num_threads(os.cpu_count())
    pipe = load_pipeline(CASE["model"], device="cpu", seed=0)
    ucfg = pipe.unet.config
    usd = {k: v.detach() for k, v in pipe.unet.state_dict().items()}
    te, vae, tok = pipe.text_encoder, pipe.vae, pipe.tokenizer
    tsd = {k: v.detach() for k, v in te.state_dict().items()}
    vsd = {k: v.detach() for k, v in vae.state_dict().items()}
    ids, nids = tok([CASE["prompt"]]), tok([""])
    lat = latents(ucfg)
    out = dict(ids=ids.numpy(), nids=nids.numpy(), lat_in=lat.numpy(),
               fp_unet=np.float64(CC.fingerprint(usd)), fp_te=np.float64(CC.fingerprint(tsd)),
               fp_vae=np.float64(CC.fingerprint(vsd)))
    vcfg = {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(vae.config).items()}
    for variant, dt in (("half", torch.float16), ("fp32", torch.float32)):
        t0 = time.time()
        m = hf_clip(te.config, tsd, dt)
        with torch.no_grad():
            ctx = torch.cat([m(input_ids=nids).last_hidden_state, m(input_ids=ids).last_hidden_state]).half()
        ts, a_t, a_p = ddim_tables(CASE["steps"])
        lref = denoise(RefUNet(CC.cfgdict(ucfg), usd, dict(CASE["qc"]), variant=variant), lat, ctx, ts, a_t, a_p,
                       CASE["guidance"])
        img = postprocess(RefVAEDecoder(vcfg, vsd, None, variant=variant).decode(lref))
        out[f"ctx_{variant}"] = ctx.numpy()
        out[f"lat_{variant}"] = lref.numpy()
        out[f"u8_{variant}"] = to_uint8(img)
        print(f"{variant}: {time.time() - t0:.1f}s, image {out[f'u8_{variant}'].shape} "
              f"mean {out[f'u8_{variant}'].mean():.2f}", flush=True)
    d = np.abs(out["u8_half"].astype(np.int16) - out["u8_fp32"].astype(np.int16))
    print(f"half vs fp32 oracle: max {d.max()} levels, mean {d.mean():.3f}, >8 levels {(d > 8).mean():.4%}")
    np.savez_compressed(OUT, **out)
    os.chmod(OUT, 0o644)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
