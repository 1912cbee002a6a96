import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "nerf-or-nothing_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnof.so on the GPU)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    if not os.path.exists(O.LIB_PATH):
        import subprocess

        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nof

    nof.lib()  # must load: no CPU fallback exists
    return torch.device("cuda", 0)


def rel_l2(a, b):
    import numpy as np

    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))
