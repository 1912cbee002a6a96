"""BASELINE configs[0] at its stated size, on the CPU reference path (the oracle): one 400x400
synthetic Lego-shaped view, 4096 rays x 64+64 samples, the 4x128 MLP (no skip, 128-wide view layer).

The reference runs this configuration only on its CPU path (MipNerfModel.GetGradient, MNcs:99-200;
TrainState.cs:25-37 for Adam), so it is the oracle's float restatement that runs here: three
training steps on one fixed batch (same samples every step), checking the sample t-values
bit-exactly against the standalone samplers and a finite, decreasing loss.
"""
import os

import numpy as np

NTHREADS = min(16, len(os.sched_getaffinity(0)))


def test_config1_fullsize_cpu_training(oracle):
    from nof import synth

    n, samples, seed = 4096, (64, 64), 0x5EED0001
    spec = oracle.Spec(D=4, W=128, Dc=1, Wc=128)
    assert oracle.param_count(spec) == int(sum(oracle.layer_sizes(spec)))  # 4x128 spec
    r = synth.blender_rays(n, width=400, height=400, num_views=1, seed=1)
    P = oracle.glorot_init(spec, seed)
    m = np.zeros_like(P)
    v = np.zeros_like(P)
    losses = []
    for it in range(1, 4):
        out = oracle.step(spec, P, r, samples=samples, seed=seed, step_idx=0, dtype=np.float32, nthreads=NTHREADS,
                          want=("t", "w", "grads"))
        # t: level 0 = the stratified sampler, level 1 = the resampler fed level 0's float weights
        t0 = oracle.sample_stratified(r["near"], r["far"], samples[0], True, seed, 0, 0, 0)
        assert np.array_equal(out["t"][0], t0)
        t1, idx = oracle.sample_pdf(out["t"][0], out["w"][0], samples[1], 0.01, True, seed, 0, 1, 0)
        assert np.array_equal(out["t"][1], t1)
        assert idx.min() >= 0 and idx.max() <= samples[0] - 1
        G = out["grads"]
        assert np.all(np.isfinite(G)) and np.isfinite(out["loss"])
        losses.append(out["loss"])
        oracle.adam_step(P, G.astype(np.float32), m, v, 5e-4, it)  # lr_init (TrainState.cs:54)
    final = oracle.step(spec, P, r, samples=samples, seed=seed, step_idx=0, dtype=np.float32, nthreads=NTHREADS,
                        want=())
    losses.append(final["loss"])
    print("config 1 losses:", losses)
    assert all(np.isfinite(losses))
    assert all(b < a for a, b in zip(losses, losses[1:])), f"loss not decreasing: {losses}"
