"""F16 forward / backward phase stamps per 256-sample group (build: python tools/diag/variant.py stamps h32_stamps).

    NOF_LIB=$PWD/build_diag/stamps/nerf-or-nothing_amd/lib/libnof.so python tools/diag/h32_stamps.py [rays]

Runs config-2-shaped F16 steps and prints, for the last k_mlp_fwd_h32 and k_mlp_bwd_h32 launch, wave 0's
mean cycles per phase of a group (s_memtime; first groups of a workgroup and later ones apart), the
launch's wall-clock span (s_memrealtime, 100 MHz) and the groups' spans."""
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
phases = {0: [("view PE + dirb", 0, 7), ("IPE", 7, 8), ("swap + act_in", 8, 9), ("first barrier", 9, 1),
              ("layer 0", 1, 2), ("layers 1-7", 2, 3), ("view layer", 3, 4), ("last tile + heads", 4, 5)],
          1: [("loads + heads", 0, 7), ("delta9 + stores", 7, 9), ("first barrier", 9, 1), ("layer 9 (dh7)", 1, 2),
              ("layers 7-2", 2, 3), ("layer 1", 3, 4), ("last tile", 4, 5)]}
ngroups = n * 128 // 256
for k in (0, 1):
    buf = (C.c_ulonglong * 131072)()
    assert lib.nof_diag_h32_stamps(buf, k) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 16)[:ngroups].astype(np.int64)
    wg = st[:, 13]
    first = np.zeros(ngroups, bool)
    for b in np.unique(wg):
        first[np.where(wg == b)[0].min()] = True
    rt0, rt1 = st[:, 14], st[:, 15]
    span_us = (rt1.max() - rt0.min()) / 100.0
    gdur = (rt1 - rt0) / 100.0
    name = "fwd" if k == 0 else "bwd"
    print(f"{name}: {ngroups} groups on {len(np.unique(wg))} workgroups, launch span {span_us:.1f} us; group "
          f"{gdur[first].mean():.1f} us first, {gdur[~first].mean() if (~first).any() else 0:.1f} us later")
    tot = (st[:, 5] - st[:, 0]).astype(float)
    for p, a_, b_ in phases[k]:
        c = (st[:, b_] - st[:, a_]).astype(float)
        f = f"{c[first].mean():9.0f} ({c[first].mean() / tot[first].mean():.3f})"
        l = f"{c[~first].mean():9.0f} ({c[~first].mean() / tot[~first].mean():.3f})" if (~first).any() else ""
        print(f"   {p:18s} first {f}   later {l}")
