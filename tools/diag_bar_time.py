"""Diagnostic (NOF_DIAG_WG_TIME + NOF_DIAG_BAR_TIME builds): fraction of each wave's lifetime the
fused MLP kernels spend in the slice barriers — waiting for the weight-slice DMA (vmcnt) and at
s_barrier for the other waves.  usage: NOF_LIB=.../libnof_bar.so python tools/diag_bar_time.py f32|f16x2"""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))
import torch
import nof
from nof import synth

prec = {"f32": 0, "split": 1, "f16x2": 2}[sys.argv[1] if len(sys.argv) > 1 else "f32"]
n = 1024
m = nof.AcceleratedMipNeRF(max_rays=n, num_samples=(128, 128), precision=prec)
r = synth.blender_rays(n, seed=1)
d = {k: torch.from_numpy(v).cuda() for k, v in r.items()}
for _ in range(5):
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
torch.cuda.synchronize()
lib = nof.lib()
for name in ("fwd", "bwd"):
    buf = (C.c_ulonglong * (4096 * 8 * 3))()
    assert getattr(lib, f"nof_diag_{name}_bar")(buf) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(4096 * 8, 3).astype(np.float64)
    t = t[t[:, 2] > 0]
    vm, bar, life = t[:, 0].sum(), t[:, 1].sum(), t[:, 2].sum()
    print(f"{name}: {len(t)} waves, mean lifetime {t[:, 2].mean():.0f} cycles; vmcnt wait {vm / life:.3f}, "
          f"s_barrier wait {bar / life:.3f} of the lifetime (per-wave barrier share p10/p50/p90 "
          f"{np.percentile(t[:, 1] / t[:, 2], 10):.3f}/{np.percentile(t[:, 1] / t[:, 2], 50):.3f}/"
          f"{np.percentile(t[:, 1] / t[:, 2], 90):.3f})")
