"""Ray generation.  CPU: the oracle's geometry (oracle/raygen.py) and the host
RecenterPoses of the C ABI bit-exact against it.  GPU: device records bit-exact vs the oracle for
Blender-style and LLFF/NDC rays, and a generated dataset feeding the gather."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import raygen as RG  # noqa: E402


def _poses(V, seed=0, llff=False):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(V):
        a = rng.normal(size=3) * (0.1 if llff else 1.0)
        # rotation from an axis-angle (Rodrigues), translation on a sphere / a small plane patch
        th = np.linalg.norm(a)
        k = a / th
        K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
        t = rng.normal(size=3) * 0.2 if llff else 4.031 * rng.normal(size=3) / 2
        out.append(np.concatenate([R.ravel(), t]))
    return np.array(out, np.float32)


def test_oracle_geometry():
    P = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0.5, -1, 2], np.float32)  # identity rotation
    rec = RG.generate(P[None], 4, 2, 2.0, 2.0, 6.0)
    # pixel (0,0): d = ((0 - 2 + .5)/2, -(0 - 1 + .5)/2, -1)
    assert np.array_equal(rec[0, 3:6], np.array([-0.75, 0.25, -1.0], np.float32))
    assert np.array_equal(rec[0, 0:3], P[9:])
    assert rec[3, 9] == 0.0  # last column: the reference's zero radius
    assert abs(rec[0, 9] - 0.5 * 2 / np.sqrt(12)) < 1e-7  # |d(x) - d(x+1)| = 1/f
    assert np.allclose(np.linalg.norm(rec[:, 6:9], axis=1), 1, atol=1e-6)
    # NDC of a forward ray through the image centre stays on the axis
    o, d = RG.to_ndc([np.float32(0)] * 3, [np.float32(0), np.float32(0), np.float32(-1)], 1.0, 1.0, 1.0)
    assert o[0] == 0 and o[1] == 0 and d[2] == 2.0


def test_recenter_poses_matches_oracle():
    import nof

    P = _poses(7, seed=3, llff=True)
    assert np.array_equal(nof.recenter_poses(P), RG.recenter_poses(P))


@pytest.mark.gpu
@pytest.mark.parametrize("ndc", [False, True])
def test_device_rays_bit_exact(gpu, ndc):
    import torch
    import nof

    V, w, h = 3, 37, 23
    P = _poses(V, seed=1, llff=ndc)
    focal = 1.2 * w if ndc else 0.5 * w / np.tan(0.5 * 0.6911112)
    imgs = torch.rand((V, h, w, 3), device=gpu)
    rec = nof.generate_rays(P, w, h, focal, 2.0, 6.0, ndc=ndc, images=imgs)
    torch.cuda.synchronize()
    ref = RG.generate(P, w, h, focal, 2.0, 6.0, ndc=ndc, images=imgs.cpu().numpy())
    got = rec.cpu().numpy()
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{len(bad)} mismatches, first {bad[:3]}: {got[tuple(bad[0])]} vs {ref[tuple(bad[0])]}"


@pytest.mark.gpu
def test_generated_dataset_batches(gpu):
    import torch
    import nof

    V, w, h = 2, 16, 12
    P = _poses(V, seed=4)
    ds = nof.RayDataset(generate=dict(poses=P, width=w, height=h, focal=20.0, near=2.0, far=6.0))
    assert len(ds) == V * w * h
    b, msum = ds.next(64, 5, 1)
    torch.cuda.synchronize()
    idx = nof.to_numpy(b["record_index"][0], (64,), np.int32)
    ref = RG.generate(P, w, h, 20.0, 2.0, 6.0)
    assert np.array_equal(nof.to_numpy(b["d"][0], (64, 3)), ref[idx, 3:6])
    assert msum == 64.0
