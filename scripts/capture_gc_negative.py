"""Negative half of tests/test_gpu_capture_gc.py: the same scenario with DenoiseLoop.capture's garbage
collector handling removed (pipeline.gc replaced by a stub) must kill the process - the round-5 abort.
Runs the scenario in a child process and reports its exit status; run it ONCE, as the LAST step of a
GPU call (an abort ends the GPU work of that call):

    python3 scripts/capture_gc_negative.py > gpurun_out/<tag>_capture_gc_negative.log 2>&1
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, types
sys.path.insert(0, %r)
import qdiff_boot  # noqa: F401
import torch
from qdiff import pipeline as P
P.gc = types.SimpleNamespace(collect=lambda *a: 0, disable=lambda: None, enable=lambda: None, isenabled=lambda: False)
sys.path.insert(0, %r)
from test_gpu_capture_gc import scenario
eager, got = scenario(torch.device("cuda:0"))
print("child finished: equal", bool(torch.equal(eager, got)))
""" % (ROOT, os.path.join(ROOT, "tests"))


def main():
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=600)
    lines = (r.stdout + r.stderr).strip().splitlines()
    cause = [l for l in lines if "rror" in l or "captur" in l.lower() or "what()" in l][:12]
    print("\n".join(["-- the child's error lines:"] + cause + ["-- the child's last lines:"] + lines[-6:]))
    print(f"child exit status {r.returncode} (expected non-zero: the capture aborts without pipeline.py's "
          f"collect-before / collector-off-during capture)")
    sys.exit(0 if r.returncode != 0 else 1)


if __name__ == "__main__":
    main()
