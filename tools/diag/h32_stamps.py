"""F16 forward / backward phase stamps (build: python tools/diag/variant.py stamps h32_stamps).

    NOF_LIB=$PWD/build_diag/stamps/nerf-or-nothing_amd/lib/libnof.so python tools/diag/h32_stamps.py [rays]

Runs config-2-shaped F16 steps and prints, for the last k_mlp_fwd_h32 and k_mlp_bwd_h32 launch, wave 0's
mean cycles per phase (s_memtime), the workgroups' wall-clock spans (s_memrealtime, 100 MHz) and how
much of launch x 256 CUs the workgroups cover."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))
import torch  # noqa: E402

import nof  # noqa: E402
from nof import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
m = nof.AcceleratedMipNeRF(max_rays=n, num_samples=(128, 128), precision=4)
r = synth.blender_rays(n, seed=1)
d = {k: torch.from_numpy(v).cuda() for k, v in r.items()}
for _ in range(5):
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
torch.cuda.synchronize()
lib = nof.lib()
names = {0: ("fwd", ["prologue", "layer 0", "layers 1-7", "view layer", "last view tile", "drain"]),
         1: ("bwd", ["prologue", "layer 9 (dh7)", "layers 7-2", "layer 1", "last tile", "drain"])}
nwg = n * 128 // 256
for k in (0, 1):
    buf = (C.c_ulonglong * 131072)()
    assert lib.nof_diag_h32_stamps(buf, k) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 16)[:nwg].astype(np.int64)
    cyc = np.diff(st[:, :7], axis=1)
    rt0, rt1 = st[:, 14], st[:, 15]
    span_us = (rt1.max() - rt0.min()) / 100.0
    dur_us = (rt1 - rt0) / 100.0
    clk = (st[:, 6] - st[:, 0]) / ((rt1 - rt0) / 100e6) / 1e9
    name, ph = names[k]
    print(f"{name}: {nwg} workgroups, launch span {span_us:.1f} us, workgroup {dur_us.mean():.1f} us "
          f"(min {dur_us.min():.1f}, max {dur_us.max():.1f}), clock {np.median(clk):.2f} GHz, "
          f"coverage {dur_us.sum() / (256 * span_us):.3f} of 256 CUs x span")
    tot = cyc.sum(axis=1).mean()
    for i, p in enumerate(ph):
        print(f"   {p:16s} {cyc[:, i].mean():9.0f} cyc  ({cyc[:, i].mean() / tot:.3f})")
    pro = ["encodings" if k == 0 else "heads", "act_in / view PE" if k == 0 else "delta9 + stores",
           "tables" if k == 0 else "w8 table", "prologue barrier"]
    pts = [0, 7, 8, 9, 1]
    for i, p in enumerate(pro):
        a_, b_ = pts[i], pts[i + 1]
        if (st[:, b_] > 0).all():
            print(f"     prologue: {p:18s} {(st[:, b_] - st[:, a_]).mean():9.0f} cyc")
        else:
            pts[i + 1] = a_
    starts = np.sort((rt0 - rt0.min()) / 100.0)
    print("   start times (us) quantiles:", np.round(np.quantile(starts, [0, .25, .5, .55, .75, 1.0]), 1))
