"""GPU evaluation path: forward-only render (MipNerfModel.Call, MNcs:36-97)
and image metrics (MipHelpers.cs:672, 685-736) against the fp64 oracle / the training path."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import metrics as M  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev(r, gpu):
    import torch

    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(gpu) for k, v in r.items()}


@pytest.mark.parametrize("precision", [0, 1, 2, 3, 4])
def test_render_equals_training_forward(gpu, oracle, precision):
    """render_device (inference kernels: no side outputs) == the forward half of the training step,
    bitwise, on the same Philox state; distance / acc match the fp64 restatement."""
    import torch
    import nof
    from nof import synth

    n, samples = 48, (64, 128)
    r = synth.blender_rays(n, seed=21)
    d = _dev(r, gpu)
    m = nof.AcceleratedMipNeRF(seed=9, max_rays=n, num_samples=samples, precision=precision)
    m.set_rng(0xABC, 4, 100)
    lv = m.render_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], randomized=True)
    torch.cuda.synchronize()
    out = [{k: nof.to_numpy(p, s) for k, (p, s) in L.items()} for L in lv]
    views = [m.level_numpy(l) for l in range(2)]
    assert m.get_rng()[1] == 4, "render must not advance the training step"
    for l in range(2):
        dist, acc = M.render_distance_acc(views[l]["weights"], views[l]["t"])
        assert np.allclose(out[l]["acc"], acc, rtol=1e-6, atol=1e-6)
        assert np.allclose(out[l]["distance"], dist, rtol=1e-6, atol=1e-5)
        assert np.array_equal(out[l]["comp_rgb"], views[l]["comp_rgb"])
    m.set_rng(0xABC, 4, 100)
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
    torch.cuda.synchronize()
    for l in range(2):
        assert np.array_equal(m.level_numpy(l)["comp_rgb"], out[l]["comp_rgb"]), f"level {l}"
    m.close()


def test_render_deterministic_grid(gpu, oracle):
    import torch
    import nof
    from nof import synth

    n = 16
    r = synth.blender_rays(n, seed=3)
    d = _dev(r, gpu)
    m = nof.AcceleratedMipNeRF(seed=1, max_rays=n, num_samples=(64, 64))
    m.render_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], randomized=False)
    torch.cuda.synchronize()
    t0 = oracle.sample_stratified(r["near"], r["far"], 64, False)
    assert np.array_equal(m.level_numpy(0)["t"], t0)
    whole = m.level_numpy(1)["comp_rgb"]
    res = m.render_rays(r, randomized=False, chunk=5)  # host chunked path == one call
    assert np.array_equal(res[1]["comp_rgb"], whole)
    m.close()


def test_image_metrics_vs_oracle(gpu):
    import nof

    rng = np.random.default_rng(7)
    a = rng.random((37, 53, 3)).astype(np.float32)
    b = np.clip(a + rng.normal(0, 0.08, a.shape), 0, 1).astype(np.float32)
    p, s = nof.image_metrics(a, b)
    assert abs(p - M.psnr(a, b)) < 1e-4
    assert abs(s - M.ssim(a, b)) < 1e-5
    p, s = nof.image_metrics(a, a)
    assert s == pytest.approx(1.0, abs=1e-6) and p > 100
