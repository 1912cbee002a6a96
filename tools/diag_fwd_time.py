"""Diagnostic (NOF_DIAG_FWD_TIME builds, not kept in the product): per-workgroup phase timestamps of
the last forward launch (wave 0 of each workgroup, wall_clock64 at 100 MHz): prologue, layer 0,
trunk 1..6, layer 7, view layer, heads; and the idle time between workgroups.
usage: NOF_LIB=.../libnof_fwdt.so python tools/diag_fwd_time.py f32|f16x2"""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))
import torch
import nof
from nof import synth
prec = {"f32": 0, "f16x2": 2, "f16split": 3}[sys.argv[1] if len(sys.argv) > 1 else "f32"]
n = 1024
m = nof.AcceleratedMipNeRF(max_rays=n, num_samples=(128, 128), precision=prec)
r = synth.blender_rays(n, seed=1)
d = {k: torch.from_numpy(v).cuda() for k, v in r.items()}
for _ in range(3):
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
torch.cuda.synchronize()
buf = (C.c_ulonglong * 8192)()
assert nof.lib().nof_diag_fwd_times(buf) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8)[:, :7].astype(np.int64)
t = t[t[:, 6] > 0]
t0 = t[:, 0].min()
us = (t - t0) / 100.0
ph = np.diff(us, axis=1)
names = ["prologue", "layer 0", "trunk 1-6", "layer 7", "view layer", "heads"]
tot = us[:, 6] - us[:, 0]
print(f"{len(t)} workgroups, launch {us[:, 6].max():.1f} us, mean workgroup {tot.mean():.1f} us, "
      f"CU-time busy {tot.sum() / (256 * us[:, 6].max()):.3f}")
for i, nm in enumerate(names):
    print(f"  {nm:11s} mean {ph[:, i].mean():8.2f} us  ({ph[:, i].mean() / tot.mean():.3f})  min {ph[:, i].min():.2f} max {ph[:, i].max():.2f}")
s = np.sort(us[:, 0])
print("start times (first 4 rounds' firsts):", np.round(s[[0, 255, 256, 511, 512, 767, 768]], 1) if len(s) >= 769 else np.round(s[:8], 1))
