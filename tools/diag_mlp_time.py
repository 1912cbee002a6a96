"""Diagnostic (NOF_DIAG_WG_TIME builds): workgroup start/end times of the last fused MLP forward and
backward launches — dispatch rounds, per-workgroup duration spread and tail (CU-time efficiency).
usage: NOF_LIB=.../libnof_wgt.so python tools/diag_mlp_time.py f32|f16x2"""
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
for _ in range(3):
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
torch.cuda.synchronize()
lib = nof.lib()
ncu = torch.cuda.get_device_properties(0).multi_processor_count
for name in ("fwd", "bwd"):
    buf = (C.c_ulonglong * 8192)()
    assert getattr(lib, f"nof_diag_{name}_times")(buf) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 2).astype(np.int64)
    t = t[t[:, 1] > 0]
    t0 = t[:, 0].min()
    s, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
    du = e - s
    span = e.max()
    print(f"{name}: {len(t)} workgroups, launch {span:.1f} us, workgroup us min/median/max "
          f"{du.min():.1f}/{np.median(du):.1f}/{du.max():.1f}; CU-time efficiency {du.sum() / (ncu * span):.3f}; "
          f"last start {s.max():.1f} us, first end {e.min():.1f} us, ends after {span - 5:.0f} us: {(e > span - 5).sum()}")
    hist, edges = np.histogram(e, bins=10)
    print("   end histogram:", list(zip(np.round(edges[:-1]).astype(int).tolist(), hist.tolist())))
