"""Kernel choice - and therefore every result - is reproducible across processes.

The GEMM tuner's choice of kernel variant changes the fp32 summation order for split-K and halo
candidates, which the W8A8 network amplifies; the committed MI355X-tuned table
(quantization---diffusion-models_amd/gemm_table.json, scripts/tune_table.py) fixes the choice for
every shape of the bench configurations.  Two fresh processes run the C2 workload (SD1.5 W8A8
SmoothQuant, 4 prompts = CFG batch 8, 3 graph-replayed DDIM steps) in both W8A8 modes: bit-identical
latents, and no shape left for either process to tune.  (The reference's CPU path is deterministic:
quantize/fake_quant.py:223, 339.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TABLE = os.path.join(os.path.dirname(HERE), "quantization---diffusion-models_amd", "gemm_table.json")


def _run(mode):
    env = dict(os.environ)
    env.pop("QD_GEMM_TABLE", None)  # the committed table
    r = subprocess.run([sys.executable, os.path.join(HERE, "helpers", "c2_latents.py"), mode], capture_output=True,
                       text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["fakequant", "int8"])
def test_two_fresh_processes_give_bit_identical_c2_latents(mode):
    assert os.path.exists(TABLE), "gemm_table.json missing: run scripts/tune_table.py on an MI355X"
    a, b = _run(mode), _run(mode)
    print(f"[determinism {mode}] {a} | {b}", flush=True)
    assert a["finite"] and b["finite"]
    assert a["table"] > 0 and a["tuned"] == 0 and b["tuned"] == 0, (a, b)
    assert a["sha256"] == b["sha256"], (a, b)
