"""Child process of tests/test_gpu_determinism.py (TEST HELPER): one fresh process builds the C2
model (SD1.5 W8A8 SmoothQuant with the fixture's activation statistics, tests/test_gpu_c2.py), runs
a 3-step CFG-batch-8 generate through the step graph and prints one JSON line: the sha256 of the
final latents' bytes, and how many GEMM shapes the process had to tune itself (0 = every kernel
choice came from the committed gemm_table.json)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402


def main():
    from test_gpu_c2 import _inputs, _sq_model
    n0 = len(K.gemm_choices())
    model, _ = _sq_model(int8_mfma=len(sys.argv) > 1 and sys.argv[1] == "int8")
    x, _, ctx = _inputs(model.pipeline.unet)
    pe, ne = ctx[4:], ctx[:4]
    lat = model.generate(prompt_embeds=pe, negative_prompt_embeds=ne, lat=x[:4], num_inference_steps=3,
                         output_type="latent").cpu()
    torch.cuda.synchronize()
    print(json.dumps({"sha256": hashlib.sha256(lat.numpy().tobytes()).hexdigest(), "tuned": len(K.gemm_choices()) - n0,
                      "table": n0, "finite": bool(torch.isfinite(lat.float()).all())}), flush=True)


if __name__ == "__main__":
    main()
