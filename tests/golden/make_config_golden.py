"""Oracle outputs at BASELINE.json's full-size configs (TEST FIXTURES; run in the build container,
whose AVX512-FP16 CPU runs the half oracle's torch-CPU Half kernels at speed):

    python tests/golden/make_config_golden.py [c1 c2 c3 c4]

For every case of oracle/config_cases.py: the synthetic checkpoint's UNet (CPU generator,
seed 0), the half and fp32 oracle results on the case's seeded inputs, and the weights'
fingerprint, into tests/golden/config_golden.safetensors (merged with the cases already there).
tests/test_gpu_configs.py compares the GPU with them.
"""
import json
import os
import sys
import time

import torch
from safetensors.torch import load_file, save_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import qdiff_boot  # noqa: E402,F401

from oracle import config_cases as CC  # noqa: E402

OUT = os.path.join(HERE, "config_golden.safetensors")


def _unet(model):
    from qdiff.unet import SD15, SDXL, UNet2DConditionModel
    cfg = SD15 if model == "sd15" else SDXL
    return cfg, UNet2DConditionModel(cfg).half().init_synthetic(0)


def main(names):
    tensors, meta = {}, {}
    if os.path.exists(OUT):
        from safetensors import safe_open
        tensors = load_file(OUT)
        with safe_open(OUT, "pt") as f:
            meta = dict(f.metadata() or {})
    torch.set_num_threads(os.cpu_count())
    built = {}
    for name in names:
        c = CC.CASES[name]
        if c["model"] not in built:
            cfg, net = _unet(c["model"])
            sd = {k: v.detach() for k, v in net.state_dict().items()}
            built[c["model"]] = (cfg, sd, CC.fingerprint(sd))
            del net
        cfg, sd, fp = built[c["model"]]
        for variant in ("half", "fp32"):
            t0 = time.time()
            y = CC.oracle_output(name, cfg, sd, variant)
            print(f"{name} {variant}: {tuple(y.shape)} in {time.time() - t0:.1f}s "
                  f"finite {bool(torch.isfinite(y.float()).all())}", flush=True)
            tensors[f"{name}.{variant}"] = y.to(torch.float16).contiguous()
        if "sq_alpha" in c:  # the SmoothQuant activation statistics the fold used
            for p, (a1, a3) in CC.sq_acts(name, cfg).items():
                tensors[f"{name}.act.{p}.norm1"] = a1.contiguous()
                tensors[f"{name}.act.{p}.norm3"] = a3.contiguous()
        meta[name] = json.dumps({"fingerprint": fp, "case": c, "threads": torch.get_num_threads()})
    save_file(tensors, OUT, metadata=meta)
    print("wrote", OUT)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CC.CASES))
