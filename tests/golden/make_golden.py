"""Regenerate tests/golden/*.npz from the independent torch/numpy restatement (tests/torch_ref.py).

    python tests/golden/make_golden.py

The fixtures pin oracle/oracle.cpp (the reference itself cannot run here and holds no vectors;
see oracle.cpp header).  Inputs come from nof.synth (deterministic) and torch_ref's own
Philox-based Glorot init; outputs are the restatement's t-values (fp32), resample indices,
per-level weights/colours, loss and gradients (fp64 autograd).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "nerf-or-nothing_amd")]
import torch_ref as TR  # noqa: E402
from nof import synth  # noqa: E402

CASES = {
    # config-1-shaped (4x128 MLP, 64 samples per level), full gradients stored
    "small_4x128": dict(net=dict(D=4, W=128, Dc=1, Wc=128), n=6, samples=(64, 64), seed=0xC0FFEE, step=5,
                        ray_base=17, param_seed=77, rays_seed=21, full_grads=True),
    # the reference network (8x256, skip at 4), two rays
    "ref_8x256": dict(net=dict(D=8, W=256, Dc=1, Wc=128), n=2, samples=(64, 64), seed=0x5EED, step=1,
                      ray_base=0, param_seed=1234, rays_seed=3, full_grads=False),
}


def make(name, c):
    net = TR.Net(**c["net"])
    P = TR.glorot(net, c["param_seed"])
    rays = synth.blender_rays(c["n"], seed=c["rays_seed"])
    res = TR.step(P, rays, samples=c["samples"], seed=c["seed"], step_idx=c["step"], ray_base=c["ray_base"], net=net)
    out = {"params_seed": np.array(c["param_seed"]), "param_checksum": np.array(float(P.astype(np.float64).sum())),
           "loss": np.array(res["loss"])}
    for k in ("o", "d", "radius", "near", "far", "lossmult", "pix"):
        out["ray_" + k] = rays[k]
    for l in range(len(c["samples"])):
        out[f"t{l}"] = res["t"][l]
        out[f"w{l}"] = res["w"][l]
        out[f"C{l}"] = res["C"][l]
        if res["idx"][l] is not None:
            out[f"idx{l}"] = res["idx"][l]
    G = res["grads"]
    sizes = [o * i for o, i in zip(net.outs, net.ins)] + list(net.outs)
    out["grad_norms"] = np.array([np.linalg.norm(g) for g in np.split(G, np.cumsum(sizes)[:-1])])
    if c["full_grads"]:
        out["grads"] = G
    else:
        rng = np.random.default_rng(0)
        idx = np.sort(rng.choice(G.size, 4096, replace=False))
        out["grad_idx"] = idx
        out["grad_vals"] = G[idx]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "loss", res["loss"], "bytes", os.path.getsize(os.path.join(HERE, name + ".npz")))


if __name__ == "__main__":
    for name, c in CASES.items():
        make(name, c)
