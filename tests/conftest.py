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


# The F16 mode's gradient bound (NOF_PRECISION_F16), per gradient tensor, relative L2 against an
# fp64 oracle that makes its OWN ReLU decisions.  Its forward rounds weights and activations to fp16 before
# every product, so units with |z| within fp16 rounding of 0 gate the other way than fp64 does; each such
# flip moves every gradient below that unit, most of all W0's (the deepest delta times the fp16 IPE).
# Measured (GPUTEST r05): W0 3.3e-3 at config 2 (1024 x 128+128), 4.9e-3 at configs[4]'s per-GPU shape
# (512 LLFF rays x 256+256), 3.1e-3 on the two-ray golden fixture; the median tensor 5e-4, the whole
# arena 2.9e-4.  With the GPU's ReLU decisions adopted the gradients are within 2e-3 (measured 5.3e-4);
# the forward outputs and the integrator adjoint are within 2e-3 without adoption.
# Per tensor (round 6): only layer 0's pair gets headroom over SURVEY §8(d)'s 2e-3
# perf-mode bound — 6e-3 for W0 (measured 4.9e-3) and b0 (2.5e-3 on the two-ray golden fixture), the two
# tensors formed from delta0, the deepest delta, which every flip above it moves — and every other tensor
# (median 5e-4) is held to 2e-3, so a regression in any of them fails.
F16_GRAD_TOL_L0 = 6e-3
F16_GRAD_TOL = 2e-3
F16_L0_TENSORS = (0, 11)  # W0, b0 in the arena order [W0..W10, b0..b10]


def f16_grad_tol(tensor):
    """the F16 mode's bound for gradient tensor `tensor` of the arena order [W0..W10, b0..b10]"""
    return F16_GRAD_TOL_L0 if tensor in F16_L0_TENSORS else F16_GRAD_TOL


def rel_l2(a, b):
    import numpy as np

    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))
