"""Diagnostic: per-tensor gradient error of one GPU step vs the fp64 oracle."""
import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nerf-or-nothing_amd"), os.path.join(ROOT, "oracle")]
import nof, oracle as O
from nof import synth
n, samples = int(sys.argv[1]), (int(sys.argv[2]), int(sys.argv[3]))
seed, step, rb = 0x1234, 3, 500
m = nof.AcceleratedMipNeRF(seed=seed, max_rays=n, num_samples=samples); m.set_rng(seed, step, rb)
r = synth.blender_rays(n, seed=11)
d = {k: torch.from_numpy(v).cuda() for k, v in r.items()}
m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(r["lossmult"].sum()))
torch.cuda.synchronize()
lv = [m.level_numpy(l) for l in range(2)]
pp, P = m.mlp.flat_params(); params = nof.to_numpy(pp, (P,)); G = nof.to_numpy(m.mlp.flat_grads()[0], (P,))
ref = O.step(O.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=rb, t_override={1: lv[1]["t"]}, nthreads=16)
off = 0
for i, s in enumerate(O.layer_sizes(O.Spec())):
    a, b = G[off:off+s], ref["grads"][off:off+s]
    print(i, s, "rel %.3g" % (np.linalg.norm(a-b)/np.linalg.norm(b)), "maxabs %.3g" % np.abs(a-b).max()); off += s
for l in range(2):
    for k in ("density", "rgb", "weights", "comp_rgb", "density_grad", "rgb_grad"):
        rk = {"density": "sigma", "weights": "w", "comp_rgb": "C", "density_grad": "dsigma", "rgb_grad": "drgb"}.get(k, k)
        a, b = lv[l][k], ref[rk][l]
        print(l, k, "rel %.3g" % (np.linalg.norm(a-b)/np.linalg.norm(b)))
