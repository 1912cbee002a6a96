"""Probe: do two independent training steps on two HIP streams overlap profitably?

Two AcceleratedMipNeRF objects (same precision), each on its own torch stream, run K gradient steps
either one after the other (serial) or interleaved launch-by-launch on the two streams (concurrent).
A concurrent/serial throughput ratio above 1 means the step's kernels have complementary bottlenecks
(e.g. the HBM-bound f16x2 weight-gradient launch beside the MFMA-bound backward) worth overlapping
inside one step.  Diagnostic only (tools/).

usage: python tools/concurrency_probe.py [precision ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import nof  # noqa: E402
from nof import synth  # noqa: E402

PRECS = {"f32": 0, "split": 1, "f16x2": 2, "f16split": 3}


def main():
    precs = sys.argv[1:] or ["f32", "f16x2", "f16split"]
    dev = torch.device("cuda", 0)
    n, K = 1024, 20
    for prec in precs:
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        models = [nof.AcceleratedMipNeRF(device=0, max_rays=n, num_samples=(128, 128), seed=7 + i,
                                         stream=s.cuda_stream, precision=PRECS[prec]) for i, s in enumerate(streams)]
        r = synth.blender_rays(n, seed=3)
        d = {k: torch.from_numpy(v).to(dev) for k, v in r.items()}
        msum = float(np.sum(r["lossmult"]))

        def step(m, k):
            m.set_rng(7, k, 0)
            m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], msum)

        for m in models:
            for k in range(3):
                step(m, k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for m in models:
            for k in range(K):
                step(m, k)
        torch.cuda.synchronize()
        serial = time.perf_counter() - t0
        t0 = time.perf_counter()
        for k in range(K):
            for m in models:
                step(m, k)
        torch.cuda.synchronize()
        conc = time.perf_counter() - t0
        print(f"{prec:9s} serial {serial * 1e3 / (2 * K):7.3f} ms/step  concurrent {conc * 1e3 / (2 * K):7.3f} ms/step  "
              f"ratio {serial / conc:.3f}", flush=True)
        for m in models:
            m.close()


if __name__ == "__main__":
    main()
