"""Bitwise A/B of two library builds: the same training steps, every output compared bit for bit.

    NOF_LIB=<lib A> python tools/ab_bits.py gpurun_out/a.npz
    NOF_LIB=<lib B> python tools/ab_bits.py gpurun_out/b.npz
    python tools/ab_bits.py --compare gpurun_out/a.npz gpurun_out/b.npz

Each run: for every precision mode, a config-2-shaped model (1024 rays x 128+128, and a 64+128 model for
the unequal-levels path) takes two training steps (get_gradient_device + Adam) on fixed synthetic batches;
the gradient arena, every level's per-ray outputs and adjoints, the loss and the parameters after Adam are
saved.  A refactoring that claims "same arithmetic" must compare equal here.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))


def run(out):
    import torch

    import nof
    from nof import synth

    dev = torch.device("cuda", 0)
    res = {}
    for prec in (0, 1, 2, 3, 4):
        for samples in ((128, 128), (64, 128)):
            n = 1024
            tag = f"p{prec}_s{samples[0]}"
            model = nof.AcceleratedMipNeRF(seed=11, max_rays=n, num_samples=samples, precision=prec)
            opt = nof.AcceleratedAdamOptimizer(model.GetLayerSizes(), model.config)
            for step in range(2):
                r = synth.blender_rays(n, seed=100 + step)
                d = {k: torch.from_numpy(v).to(dev) for k, v in r.items()}
                model.set_rng(0x5EED0A0B, step, 0)
                grads = model.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"],
                                                  d["pix"], float(np.sum(r["lossmult"], dtype=np.float32)))
                torch.cuda.synchronize()
                G = nof.to_numpy(model.mlp.flat_grads()[0], (546948,)).copy()
                res[f"{tag}_grads{step}"] = G
                res[f"{tag}_loss{step}"] = np.float32(model.loss())
                for l in range(2):
                    lv = model.level_numpy(l)
                    for k in ("t", "weights", "comp_rgb", "density_grad", "rgb_grad"):
                        res[f"{tag}_{k}{l}_{step}"] = lv[k].copy()
                opt.step(model.mlp.allParams, grads, nof.learning_rate_decay(step + 1))
                torch.cuda.synchronize()
            res[f"{tag}_params"] = nof.to_numpy(model.mlp.flat_params()[0], (546948,)).copy()
            model.close()
    np.savez(out, **res)
    print(f"{out}: {len(res)} arrays")


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if k not in B.files or A[k].tobytes() != B[k].tobytes()]
    for k in bad[:20]:
        x, y = A[k].astype(np.float64), B[k].astype(np.float64)
        print(f"DIFF {k}: rel L2 {np.linalg.norm(x - y) / max(np.linalg.norm(x), 1e-300):.3g}")
    print(f"{len(A.files) - len(bad)} / {len(A.files)} arrays bitwise equal")
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
