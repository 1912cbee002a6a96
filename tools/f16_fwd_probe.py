"""F16 forward with and without its side outputs (k_mlp_fwd_h32<true> in the training step vs <false> in
render_device), same rays, for rocprofv3 --kernel-trace --stats: the store stream's share of the forward.

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run --output-format csv -- python tools/f16_fwd_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))


def main():
    import torch
    import nof
    from nof import synth

    n = 1024
    dev = torch.device("cuda", 0)
    r = {k: torch.from_numpy(v).to(dev) for k, v in synth.blender_rays(n, seed=1).items()}
    m = nof.AcceleratedMipNeRF(max_rays=n, num_samples=(128, 128), seed=3, precision=4)
    for k in range(20):
        m.set_rng(3, k, 0)
        m.get_gradient_device(n, r["o"], r["d"], r["radius"], r["near"], r["far"], r["lossmult"], r["pix"], float(n))
    for k in range(20):
        m.render_device(n, r["o"], r["d"], r["radius"], r["near"], r["far"], randomized=True)
    torch.cuda.synchronize()
    print("done", flush=True)
    m.close()


if __name__ == "__main__":
    main()
