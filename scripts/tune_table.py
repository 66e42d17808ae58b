"""Tune the GEMM kernel table on an MI355X and write it to
quantization---diffusion-models_amd/gemm_table.json (loaded by kernels.py at import: every process
that shares it runs the same kernel variant per GEMM shape, hence the same fp32 summation order and
bit-identical results - VERDICT r2 #7).

Every GEMM / conv shape of the bench configurations is met once in eager mode (the tuner times
the candidates at the first eager call of each shape): SD1.5 W8A8-SQ fake-quant and int8-MFMA
(SmoothQuant calibration at CFG batch 16, the denoising loop at CFG batch 8, CLIP + VAE), SD1.5
W4A16 at CFG batch 16 (config C3), SDXL W8A8 1024^2 (C4), SD3.5-Large W4A16 and W4A8-fp8 1024^2
(C5), and the test suite's C1 / C2 / C3 / C4 workloads.

usage (on the GPU box):  QD_GEMM_TABLE=none python scripts/tune_table.py [--models sd15,sdxl,sd35]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("QD_GEMM_TABLE", "none")   # start from an empty table
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402

OUT = os.path.join(ROOT, "quantization---diffusion-models_amd", "gemm_table.json")


def log(msg, t0=[time.time()]):
    print(f"[tune +{time.time() - t0[0]:.0f}s] {msg} ({len(K.gemm_choices())} shapes)", flush=True)


def run_sd15(dev):
    from qdiff.models import StableDiffusion1_x
    g = torch.Generator().manual_seed(0)
    prompts = [f"tuning prompt {i}" for i in range(4)]
    for mode, i8 in (("w8a8-sq", False), ("w8a8-sq-int8", True)):
        m = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
        # SmoothQuant calibration shapes (CFG batch 16), then the loop at CFG batch 8 (+ CLIP / VAE)
        m.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantType="sq",
                   quantUnet=True, int8_mfma=i8, calibration=dict(n_samples=8, batch_size=8, num_inference_steps=2))
        lat = torch.randn(4, 4, 64, 64, generator=g).half()
        m.generate(prompt=prompts, lat=lat, num_inference_steps=2, use_graph=False)
        # the CFG-batch-2 (C1) and -16 (C3) loops of the fake-quant model
        m.generate(prompt=prompts[:1], lat=lat[:1], num_inference_steps=2, use_graph=False, output_type="latent")
        log(f"sd15 {mode}")
        del m
        torch.cuda.empty_cache()
    for qc in (dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False),
               dict(w_bit=8, a_bit=16, q_group_size=128, quantize_act=False)):
        m = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
        m.quantize(quant_config=dict(qc), quantUnet=True)
        for b in (1, 8):
            lat = torch.randn(b, 4, 64, 64, generator=g).half()
            m.generate(prompt=[f"p{i}" for i in range(b)], lat=lat, num_inference_steps=2, use_graph=False,
                       output_type="latent")
        log(f"sd15 w{qc['w_bit']}a16")
        del m
        torch.cuda.empty_cache()


def run_sdxl(dev):
    from qdiff.models import StableDiffusionXL
    m = StableDiffusionXL.from_pretrained("synthetic:sdxl", device=dev, seed=0)
    m.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(2, 4, 128, 128, generator=g).half()
    m.generate(prompt=["a", "b"], lat=lat, height=1024, width=1024, num_inference_steps=2, use_graph=False)
    log("sdxl w8a8")
    del m
    torch.cuda.empty_cache()


def run_sd35(dev):
    from qdiff.models import StableDiffusion3_5
    for fp8 in (False, True):
        m = StableDiffusion3_5.from_pretrained("synthetic:sd35", device=dev, seed=0)
        m.quantize(quant_config=dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False), quantTransformer=True,
                   fp8_act=fp8)
        g = torch.Generator().manual_seed(0)
        lat = torch.randn(1, 16, 128, 128, generator=g).half()
        m.generate(prompt=["a"], lat=lat, height=1024, width=1024, num_inference_steps=2, use_graph=False,
                   output_type="latent")
        log(f"sd35 w4a{'8-fp8' if fp8 else '16'}")
        del m
        torch.cuda.empty_cache()


def run_w4(dev):
    """Only the packed-int4 (W4A16) GEMM shapes: SD1.5 at CFG batch 2 / 16, SD3.5-L."""
    from qdiff.models import StableDiffusion1_x, StableDiffusion3_5
    g = torch.Generator().manual_seed(0)
    m = StableDiffusion1_x.from_pretrained("synthetic:sd15", device=dev, seed=0)
    m.quantize(quant_config=dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False), quantUnet=True)
    for b in (1, 8):
        lat = torch.randn(b, 4, 64, 64, generator=g).half()
        m.generate(prompt=[f"p{i}" for i in range(b)], lat=lat, num_inference_steps=2, use_graph=False,
                   output_type="latent")
    log("sd15 w4a16")
    del m
    torch.cuda.empty_cache()
    m = StableDiffusion3_5.from_pretrained("synthetic:sd35", device=dev, seed=0)
    m.quantize(quant_config=dict(w_bit=4, a_bit=16, q_group_size=128, quantize_act=False), quantTransformer=True)
    lat = torch.randn(1, 16, 128, 128, generator=g).half()
    m.generate(prompt=["a"], lat=lat, height=1024, width=1024, num_inference_steps=2, use_graph=False,
               output_type="latent")
    log("sd35 w4a16")
    del m
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="sd15,sdxl,sd35")
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--add", action="store_true",
                    help="keep the committed table, tune only the shapes it lacks (new epilogue keys)")
    ap.add_argument("--drop-epi", type=int, default=0,
                    help="with --add: first drop the entries whose epilogue flags intersect this mask")
    ap.add_argument("--drop-conv-hw", type=int, default=0,
                    help="with --add: also drop the fp16 / int8 conv entries whose input side is <= this")
    ap.add_argument("--drop-all", action="store_true",
                    help="with --add: re-tune every shape the runs meet (the others keep their committed choice)")
    ap.add_argument("--drop-f16-halo-hw", type=int, default=0,
                    help="with --add: also drop the fp16 3x3 stride-1 conv entries whose input side is <= this "
                         "(new halo candidates: the 128-pixel tiles 204 / 205)")
    ap.add_argument("--retune-i8-linear", action="store_true",
                    help="keep the committed table, re-tune only the int8 linears (SD1.5, both modes run)")
    ap.add_argument("--retune-f16-linear", action="store_true",
                    help="keep the committed table, re-tune only the fp16-path linears without int4 operands "
                         "(SD1.5, both modes run)")
    ap.add_argument("--retune-f16-conv", action="store_true",
                    help="keep the committed table, re-tune only the fp16-path convs (SD1.5, both modes run)")
    ap.add_argument("--retune-i8-conv", action="store_true",
                    help="keep the committed table, re-tune only the int8 convs (SD1.5, both modes run)")
    ap.add_argument("--retune-i4", action="store_true",
                    help="keep the committed table, re-tune only the linears whose operands include packed int4")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.retune_i8_linear:
        K.load_table(OUT)
        dropped = {k: K._TUNE.pop(k) for k in [k for k in K.gemm_choices() if k[0] == "linear_i8"]}
        log(f"committed table without its {len(dropped)} int8 linears")
        run_sd15(dev)
        for key, ch in dropped.items():  # shapes this run does not meet keep their committed choice
            K._TUNE.setdefault(key, ch)
    elif a.retune_f16_linear:
        K.load_table(OUT)
        dropped = {k: K._TUNE.pop(k) for k in [k for k in K.gemm_choices() if k[0] == "linear" and "i4" not in k[-1]]}
        log(f"committed table without its {len(dropped)} fp16-path linears")
        run_sd15(dev)
        for key, ch in dropped.items():  # shapes this run does not meet keep their committed choice
            K._TUNE.setdefault(key, ch)
    elif a.retune_f16_conv:
        K.load_table(OUT)
        dropped = {k: K._TUNE.pop(k) for k in [k for k in K.gemm_choices() if k[0] == "conv"]}
        log(f"committed table without its {len(dropped)} fp16-path convs")
        run_sd15(dev)
        for key, ch in dropped.items():  # shapes this run does not meet keep their committed choice
            K._TUNE.setdefault(key, ch)
    elif a.retune_i8_conv:
        K.load_table(OUT)
        dropped = {k: K._TUNE.pop(k) for k in [k for k in K.gemm_choices() if k[0] == "conv_i8"]}
        log(f"committed table without its {len(dropped)} int8 convs")
        run_sd15(dev)
        for key, ch in dropped.items():  # shapes this run does not meet keep their committed choice
            K._TUNE.setdefault(key, ch)
    elif a.retune_i4:
        K.load_table(OUT)
        for key in [k for k in K.gemm_choices() if k[0] == "linear" and "i4" in k[-1]]:
            del K._TUNE[key]
        log("committed table without its int4 linears")
        for codes_only in (False, True):  # both W4 operand policies (their keys differ)
            K.W4_CODES_ONLY = codes_only
            run_w4(dev)
    elif a.add:
        n0 = K.load_table(OUT)
        dropped = {}
        if a.drop_epi:
            for key in [k for k in K.gemm_choices() if k[0] in ("conv_i8", "linear_i8") and
                        (k[11] if k[0] == "conv_i8" else k[5]) & a.drop_epi]:
                dropped[key] = K._TUNE.pop(key)
        if a.drop_conv_hw:
            for key in [k for k in K.gemm_choices() if k[0] in ("conv", "conv_i8") and k[2] <= a.drop_conv_hw]:
                dropped[key] = K._TUNE.pop(key)
        if a.drop_all:
            dropped.update({k: K._TUNE.pop(k) for k in list(K.gemm_choices())})
        if a.drop_f16_halo_hw:
            for key in [k for k in K.gemm_choices() if k[0] == "conv" and k[6] == 3 and k[8] == 1 and
                        k[2] <= a.drop_f16_halo_hw]:
                dropped[key] = K._TUNE.pop(key)
        log(f"committed table ({n0} shapes)")
        for name in a.models.split(","):
            {"sd15": run_sd15, "sdxl": run_sdxl, "sd35": run_sd35}[name](dev)
        for key, ch in dropped.items():  # shapes these runs do not meet keep their committed choice
            K._TUNE.setdefault(key, ch)
    else:
        for name in a.models.split(","):
            {"sd15": run_sd15, "sdxl": run_sdxl, "sd35": run_sd35}[name](dev)
        K.W4_CODES_ONLY = True  # the QD_W4_OPERAND=codes policy's int4 linears (their own keys)
        run_w4(dev)
    K.save_table(a.out)
    log(f"wrote {a.out}")


if __name__ == "__main__":
    main()
