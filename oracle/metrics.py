"""CPU oracle for the evaluation path (TEST INFRASTRUCTURE ONLY — never imported by the product).

Restates, in float64 numpy:
  * MathHelpers.MseToPsnr            ScratchNerf/MipHelpers.cs:672
  * MathHelpers.ComputeSsim/Average  ScratchNerf/MipHelpers.cs:685-736 (filter :737-753)
  * VectorImage.Convolve             ScratchNerf/MipHelpers.cs:903-927 (zero-padded 'same')
  * VolumetricRendering distance/acc ScratchNerf/MipHelpers.cs:472-492
Images are [H][W][3] (the reference's VectorImage is [x, y]; the 2-D Gaussian is symmetric, so the
orientation does not change any value).  Parity unpinned against the reference itself (C#, not
runnable here); pinned by known answers in tests/test_metrics.py.
"""
import numpy as np


def mse_to_psnr(mse):
    return -10.0 / np.log(10.0) * np.log(mse)  # MipHelpers.cs:672


def gaussian_filter(size=11, sigma=1.5):
    half = size // 2
    i = np.arange(size, dtype=np.float64) - half
    f = np.exp(-(i[:, None] ** 2 + i[None, :] ** 2) / (2 * sigma * sigma))  # MipHelpers.cs:744-747
    return f / f.sum()


def convolve_same(img, filt):
    """Zero-padded correlation, output the size of img (MipHelpers.cs:903-927)."""
    H, W = img.shape[:2]
    k = filt.shape[0]
    p = k // 2
    pad = np.zeros((H + 2 * p, W + 2 * p) + img.shape[2:], dtype=np.float64)
    pad[p:p + H, p:p + W] = img
    out = np.zeros_like(img, dtype=np.float64)
    for ky in range(k):
        for kx in range(k):
            out += pad[ky:ky + H, kx:kx + W] * filt[ky, kx]
    return out


def ssim(img0, img1, max_val=1.0, size=11, sigma=1.5, k1=0.01, k2=0.03):
    a = np.asarray(img0, np.float64)
    b = np.asarray(img1, np.float64)
    f = gaussian_filter(size, sigma)
    mu0, mu1 = convolve_same(a, f), convolve_same(b, f)
    mu00, mu11, mu01 = mu0 * mu0, mu1 * mu1, mu0 * mu1
    s00 = np.maximum(convolve_same(a * a, f) - mu00, 0)
    s11 = np.maximum(convolve_same(b * b, f) - mu11, 0)
    s01 = np.maximum(convolve_same(a * b, f) - mu01, 0)  # the reference clips the covariance too (:708)
    c1, c2 = (k1 * max_val) ** 2, (k2 * max_val) ** 2
    m = ((2 * mu01 + c1) * (2 * s01 + c2)) / ((mu00 + mu11 + c1) * (s00 + s11 + c2))
    return float(m.mean(axis=2).mean())  # ComputeSsimAverage: channel mean, then pixel mean (:726-735)


def psnr(img0, img1):
    d = np.asarray(img0, np.float64) - np.asarray(img1, np.float64)
    return float(mse_to_psnr(np.mean(d * d)))


def render_distance_acc(w, t):
    """acc = sum w; distance = clamp(sum w (t_i + t_{i+1}) / 2 / acc, t_0, t_S) (MipHelpers.cs:487-490)."""
    w = np.asarray(w, np.float64)
    t = np.asarray(t, np.float64)
    acc = w.sum(1)
    mid = w * (t[:, :-1] + t[:, 1:]) / 2
    with np.errstate(divide="ignore", invalid="ignore"):
        dist = np.where(acc > 0, mid.sum(1) / np.where(acc > 0, acc, 1), np.inf)
    return np.clip(dist, t[:, 0], t[:, -1]), acc
