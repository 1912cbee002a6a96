"""Debug: f16x2 act blocks vs the fp32 mode's (same params, same rays): NaN/inf census and error."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nerf-or-nothing_amd"))
import numpy as np, torch
import nof
from nof import synth
n, S = 16, 64
r = synth.blender_rays(n, seed=11)
d = {k: torch.from_numpy(v).cuda() for k, v in r.items()}
outs = {}
for prec in (0, 2):
    m = nof.AcceleratedMipNeRF(seed=5, max_rays=n, num_samples=(S, S), precision=prec)
    m.set_rng(1, 0, 0)
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
    torch.cuda.synchronize()
    dv = m.mlp.debug_view(0)
    M = dv["M"]
    if prec == 0:
        a = nof.to_numpy(dv["act_h"], (8, M // 32, 256, 32), np.float32)
    else:
        a = nof.to_numpy(dv["act_h"], (8, M // 32, 256, 32), np.float16).astype(np.float32)
    outs[prec] = a
    g = nof.to_numpy(m.mlp.flat_grads()[0], (546948,))
    print("prec", prec, "grad nan", np.isnan(g).sum(), "act nan", np.isnan(a).sum(), "act inf", np.isinf(a).sum())
    m.close()
# the block layouts differ (fp32: chunk XOR f%8 on 4-sample chunks; f16: XOR (f>>2)&3 on 8-sample chunks):
# compare per (layer, block, feature) sorted sample values
a0, a2 = outs[0], outs[2]
for l in range(8):
    s0 = np.sort(a0[l], axis=-1); s2 = np.sort(a2[l], axis=-1)
    bad = ~np.isclose(s0, s2, rtol=2e-3, atol=1e-3)
    print("layer", l, "mismatch", int(bad.sum()), "of", bad.size, "max", float(np.nanmax(np.abs(s0 - s2))))
    if bad.any():
        b, f, s = np.argwhere(bad)[0]
        print("  first bad block", b, "feature", f, s0[b, f][:8], s2[b, f][:8])
