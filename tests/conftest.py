import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qdiff_boot  # noqa: E402,F401  (registers the package as `qdiff`)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size (SD1.5) parity case, minutes of CPU oracle time")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return {name: np.load(os.path.join(GOLDEN, name + ".npz"))
            for name in ("fake_quant_golden", "smooth_golden", "install_golden")}


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
