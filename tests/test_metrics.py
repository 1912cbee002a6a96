"""CPU tests of the evaluation-path oracle (oracle/metrics.py): known answers for PSNR
(MipHelpers.cs:672), the reference's SSIM (MipHelpers.cs:685-736) and the render distance/acc
(MipHelpers.cs:472-492)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import metrics as M  # noqa: E402


def test_gaussian_filter_normalised_symmetric():
    f = M.gaussian_filter()
    assert f.shape == (11, 11) and abs(f.sum() - 1) < 1e-15
    assert np.allclose(f, f.T) and np.allclose(f, f[::-1, ::-1])
    assert f[5, 5] == f.max()


def test_psnr_known_answer():
    rng = np.random.default_rng(0)
    a = rng.random((20, 30, 3))
    assert abs(M.psnr(a, a + 0.1) - 20.0) < 1e-9
    assert abs(M.mse_to_psnr(1e-3) - 30.0) < 1e-12


def test_ssim_identity_and_monotone():
    rng = np.random.default_rng(1)
    a = rng.random((40, 32, 3))
    assert abs(M.ssim(a, a) - 1.0) < 1e-12
    s1 = M.ssim(a, np.clip(a + rng.normal(0, 0.05, a.shape), 0, 1))
    s2 = M.ssim(a, np.clip(a + rng.normal(0, 0.2, a.shape), 0, 1))
    assert 1.0 > s1 > s2 > 0.0


def test_convolve_same_zero_padding():
    img = np.ones((15, 15, 3))
    out = M.convolve_same(img, M.gaussian_filter())
    assert np.allclose(out[5:10, 5:10], 1.0)  # interior: full window
    assert out[0, 0, 0] < out[0, 7, 0] < out[7, 7, 0]  # corners see only a quarter of the window


def test_render_distance_acc():
    t = np.array([[2.0, 3.0, 4.0, 5.0]])
    w = np.array([[0.5, 0.25, 0.0]])
    d, acc = M.render_distance_acc(w, t)
    assert acc[0] == 0.75 and abs(d[0] - (0.5 * 2.5 + 0.25 * 3.5) / 0.75) < 1e-15
    d, acc = M.render_distance_acc(np.zeros((1, 3)), t)  # empty ray: +inf clamped to t_S
    assert acc[0] == 0 and d[0] == 5.0
