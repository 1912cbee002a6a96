"""Device-side bounds checks (include/nof.h nof_device_checks) in the checked build,
lib/libnof_check.so: the self-test bit proves the plumbing; a training step in every precision mode
(fused two-level step, bucketed weight gradients, Adam), a device dataset gather and a render fail
no check.  Runs in a child process (NOF_LIB selects the library; the parent has libnof.so loaded)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
import nof
from nof import synth
assert nof._lib.LIB_PATH.endswith("libnof_check.so"), nof._lib.LIB_PATH
dev = torch.device("cuda", 0)
assert nof.device_checks(clear=True) == 0
nof.device_checks_selftest()
bits = nof.device_checks(clear=True)
assert bits == 1 << 31, hex(bits)
assert nof.device_checks(clear=True) == 0
ds = nof.RayDataset(records=synth.pack_records(synth.blender_rays(5000, seed=3)), device=0)
for prec in (0, 1, 2, 3, 4):
    for n, samples in ((96, (64, 128)), (8, (256, 256))):
        m = nof.AcceleratedMipNeRF(seed=5, max_rays=n, num_samples=samples, precision=prec)
        opt = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)
        b, msum = ds.next(n, 7, 1, 0, None)
        p = {k: v[0] for k, v in b.items()}
        m.set_rng(7, 1, 0)
        g = m.get_gradient_device(n, p["o"], p["d"], p["radius"], p["near"], p["far"], p["lossmult"], p["pix"], msum)
        opt.step(m.mlp.allParams, g, nof.learning_rate_decay(1))
        lv = m.render_device(n, p["o"], p["d"], p["radius"], p["near"], p["far"], randomized=True)
        torch.cuda.synchronize()
        bits = nof.device_checks(clear=True)
        assert bits == 0, f"precision {prec} samples {samples}: failed checks {bits:#x}"
        opt.close(); m.close()
print("OK")
"""


def test_checked_build_runs_clean(gpu):
    lib = os.path.join(ROOT, "nerf-or-nothing_amd", "lib", "libnof_check.so")
    assert os.path.exists(lib), "build it with: make -C nerf-or-nothing_amd check"
    env = dict(os.environ, NOF_LIB=lib)
    out = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "nerf-or-nothing_amd")],
                         capture_output=True, text=True, timeout=150, env=env)
    assert out.returncode == 0 and "OK" in out.stdout, out.stdout[-2000:] + out.stderr[-3000:]
