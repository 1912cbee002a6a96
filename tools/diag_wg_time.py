"""Diagnostic (stamps builds: make STAMPS=1 -> lib/libnof_stamps.so): per-workgroup start/end spread of the last weight-gradient
launch — how well the host's cost-balanced item schedule finishes all CUs together.
usage: NOF_LIB=$PWD/nerf-or-nothing_amd/lib/libnof_stamps.so python tools/diag_wg_time.py f32|f16x2"""
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
buf = (C.c_ulonglong * 2048)()
assert lib.nof_diag_wg_times(buf, 0 if prec == 0 else 1) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 2).astype(np.int64)
t = t[t[:, 1] > 0]
t0 = t[:, 0].min()
start, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # wall_clock64 = 100 MHz -> us
dur = end - start
print(f"{len(t)} workgroups: launch {end.max():.1f} us; start spread {start.max() - start.min():.1f} us; "
      f"end min/median/max {end.min():.1f}/{np.median(end):.1f}/{end.max():.1f} us; "
      f"busy fraction {dur.sum() / (len(t) * end.max()):.3f}")
order = np.argsort(end)
print("earliest ends:", np.round(end[order[:8]], 1), " latest:", np.round(end[order[-8:]], 1))
