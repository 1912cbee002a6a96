"""K training steps of BASELINE configs[0] (4096 rays x 64+64 samples, 4x128 MLP) on the any-shape fp32
path, for rocprofv3 kernel traces of generic.hip:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gen -- python tools/generic_steps.py --steps 20

Prints ms/step (hipEvent-free wall clock over synchronised steps)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--rays", type=int, default=4096)
    p.add_argument("--samples", type=int, nargs="+", default=[64, 64])
    a = p.parse_args()
    import torch
    import nof
    from nof import synth
    from bench import CONFIG0_NET

    dev = torch.device("cuda", 0)
    n = a.rays
    r = {k: torch.from_numpy(v).to(dev) for k, v in synth.blender_rays(n, seed=1).items()}
    m = nof.AcceleratedMipNeRF(max_rays=n, num_samples=a.samples, seed=3, **CONFIG0_NET)
    adam = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)

    def step(k):
        m.set_rng(3, k, 0)
        g = m.get_gradient_device(n, r["o"], r["d"], r["radius"], r["near"], r["far"], r["lossmult"], r["pix"], float(n))
        adam.step(m.mlp.allParams, g, nof.learning_rate_decay(k + 1))

    for k in range(3):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(3, 3 + a.steps):
        step(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(f"configs[0] any-shape path: {dt * 1e3:.3f} ms/step, {n / dt:.0f} rays/s, loss {m.loss():.5f}", flush=True)
    adam.close()
    m.close()


if __name__ == "__main__":
    main()
