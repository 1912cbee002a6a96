"""Synthetic ray batches shaped like the reference's training data.

The reference's loaders cannot be used (Blender throws NotImplemented at
Dataset.cs:211; LLFF needs Windows System.Drawing; the .bin dataset is a local
file, Program.cs:23), and there is no network.  These generators reproduce the
*shape* of the data: pinhole rays per ``Dataset.GenerateRays`` (Dataset.cs:111-176)
— unnormalised directions d = R·((x−W/2+.5)/f, −(y−H/2+.5)/f, −1), radii
‖d(x,y) − d(x+1,y)‖·2/√12 — the LLFF NDC warp (``ConvertToNdc`` Dataset.cs:295-308,
radii Dataset.cs:282-289), and the 64-byte BinDataset record
{o3, d3, viewdir3, radius, near, far, lossmult, rgb3} (BinDataset.cs:40-49).
Pixel colours come from a smooth analytic field so PSNR is meaningful.

Everything is deterministic in ``seed`` and uses numpy only.
"""
from __future__ import annotations

import numpy as np

BLENDER_CAMERA_ANGLE_X = 0.6911112  # the Blender-synthetic convention (build's choice)


def _look_at(eye: np.ndarray) -> np.ndarray:
    """camera-to-world rotation looking from ``eye`` at the origin (OpenGL: camera looks down −z)."""
    fwd = -eye / np.linalg.norm(eye)
    up = np.array([0.0, 0.0, 1.0])
    if abs(np.dot(fwd, up)) > 0.99:
        up = np.array([0.0, 1.0, 0.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    true_up = np.cross(right, fwd)
    return np.stack([right, true_up, -fwd], axis=1)  # columns: x, y, z axes of the camera


def _pixel_colour(o: np.ndarray, d: np.ndarray) -> np.ndarray:
    """Smooth analytic 'scene' colour for a ray, in [0, 1]."""
    dn = d / np.linalg.norm(d, axis=-1, keepdims=True)
    p = o + 4.0 * dn
    r = 0.5 + 0.5 * np.sin(1.7 * p[..., 0] + 0.3 * p[..., 2])
    g = 0.5 + 0.5 * np.sin(1.3 * p[..., 1] - 0.7 * p[..., 0] + 1.0)
    b = 0.5 + 0.5 * np.cos(0.9 * p[..., 2] + 0.5 * p[..., 1])
    return np.stack([r, g, b], -1)


def blender_rays(n: int, width: int = 800, height: int = 800, num_views: int = 100, seed: int = 0,
                 views=None, near: float = 2.0, far: float = 6.0) -> dict:
    """``n`` random pixels (with replacement, BinDataset.cs:34) from ``num_views`` poses on a
    sphere of radius 4.031 looking at the origin.  ``views`` restricts the pool (for sharding by view).
    Returns float32 SoA: o[n,3], d[n,3], viewdir[n,3], radius[n], near[n], far[n], lossmult[n], pix[n,3]."""
    rng = np.random.default_rng(seed)
    focal = 0.5 * width / np.tan(0.5 * BLENDER_CAMERA_ANGLE_X)
    pool = np.arange(num_views) if views is None else np.asarray(views)
    vidx = pool[rng.integers(0, len(pool), n)]
    xs = rng.integers(0, width, n)
    ys = rng.integers(0, height, n)
    # deterministic poses: golden-angle spiral over the upper hemisphere
    k = np.arange(num_views)
    theta = np.arccos(1 - (k + 0.5) / num_views)  # polar angle in (0, pi/2)
    phi = k * np.pi * (3 - np.sqrt(5))
    eyes = 4.031 * np.stack([np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi), np.cos(theta)], 1)
    rots = np.stack([_look_at(e) for e in eyes])
    R = rots[vidx]
    o = eyes[vidx]

    def cam_dir(x, y):
        return np.stack([(x - width * 0.5 + 0.5) / focal, -(y - height * 0.5 + 0.5) / focal, -np.ones_like(x, float)], -1)

    d = np.einsum("nij,nj->ni", R, cam_dir(xs.astype(float), ys.astype(float)))
    nx = np.where(xs < width - 1, xs + 1, xs).astype(float)
    dn = np.einsum("nij,nj->ni", R, cam_dir(nx, ys.astype(float)))
    radius = np.linalg.norm(d - dn, axis=-1) * 2 / np.sqrt(12)
    # the last column has no right neighbour (Dataset.cs:147-151 uses x itself -> 0); mimic with the left one
    edge = xs >= width - 1
    if edge.any():
        dl = np.einsum("nij,nj->ni", R[edge], cam_dir((xs[edge] - 1).astype(float), ys[edge].astype(float)))
        radius[edge] = np.linalg.norm(d[edge] - dl, axis=-1) * 2 / np.sqrt(12)
    viewdir = d / np.linalg.norm(d, axis=-1, keepdims=True)
    pix = _pixel_colour(o, d)
    f32 = np.float32
    return {
        "o": o.astype(f32), "d": d.astype(f32), "viewdir": viewdir.astype(f32), "radius": radius.astype(f32),
        "near": np.full(n, near, f32), "far": np.full(n, far, f32), "lossmult": np.ones(n, f32),
        "pix": pix.astype(f32),
    }


def to_ndc(o: np.ndarray, d: np.ndarray, focal: float, w: float, h: float, near: float = 1.0):
    """ConvertToNdc (Dataset.cs:295-308), vectorised, float64 math."""
    t = -(near + o[:, 2]) / d[:, 2]
    o = o + t[:, None] * d
    o0 = -(2 * focal / w) * (o[:, 0] / o[:, 2])
    o1 = -(2 * focal / h) * (o[:, 1] / o[:, 2])
    o2 = 1 + 2 * near / o[:, 2]
    d0 = -(2 * focal / w) * (d[:, 0] / d[:, 2] - o[:, 0] / o[:, 2])
    d1 = -(2 * focal / h) * (d[:, 1] / d[:, 2] - o[:, 1] / o[:, 2])
    d2 = -2 * near / o[:, 2]
    return np.stack([o0, o1, o2], 1), np.stack([d0, d1, d2], 1)


def llff_rays(n: int, width: int = 800, height: int = 800, num_views: int = 20, seed: int = 0,
              near: float = 2.0, far: float = 6.0) -> dict:
    """Forward-facing LLFF-shaped batch: poses on a small plane patch looking down −z, NDC-warped
    (Dataset.cs:268-293; near/far 2/6 as the reference sets them, Dataset.cs:290-291)."""
    rng = np.random.default_rng(seed)
    focal = 1.2 * width
    v = rng.integers(0, num_views, n)
    xs = rng.integers(1, width - 1, n).astype(float)
    ys = rng.integers(1, height - 1, n).astype(float)
    offs = np.stack([0.3 * np.cos(np.arange(num_views)), 0.2 * np.sin(np.arange(num_views)), np.zeros(num_views)], 1)
    o = offs[v] + np.array([0.0, 0.0, 0.0])

    def cam(x, y):
        return np.stack([(x - width * 0.5 + 0.5) / focal, -(y - height * 0.5 + 0.5) / focal, -np.ones_like(x)], -1)

    d = cam(xs, ys)
    on, dn = to_ndc(o, d, focal, width, height)
    ox, _ = to_ndc(o, cam(xs + 1, ys), focal, width, height)
    oy, _ = to_ndc(o, cam(xs, ys + 1), focal, width, height)
    dx = np.linalg.norm(on - ox, axis=-1)
    dy = np.linalg.norm(on - oy, axis=-1)
    radius = np.sqrt(dx * dx + dy * dy) / np.sqrt(12)
    pix = _pixel_colour(o, d)
    f32 = np.float32
    return {
        "o": on.astype(f32), "d": dn.astype(f32), "viewdir": (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(f32),
        "radius": radius.astype(f32), "near": np.full(n, near, f32), "far": np.full(n, far, f32),
        "lossmult": np.ones(n, f32), "pix": pix.astype(f32),
    }


RECORD_FLOATS = 16  # BinDataset.cs:35-49: 64-byte records


def pack_records(rays: dict) -> np.ndarray:
    """SoA → BinDataset record array [n, 16] float32 (o, d, viewdir, radius, near, far, lossmult, rgb)."""
    n = rays["o"].shape[0]
    rec = np.zeros((n, RECORD_FLOATS), np.float32)
    rec[:, 0:3], rec[:, 3:6], rec[:, 6:9] = rays["o"], rays["d"], rays["viewdir"]
    rec[:, 9], rec[:, 10], rec[:, 11], rec[:, 12] = rays["radius"], rays["near"], rays["far"], rays["lossmult"]
    rec[:, 13:16] = rays["pix"]
    return rec


def unpack_records(rec: np.ndarray) -> dict:
    rec = np.asarray(rec, np.float32).reshape(-1, RECORD_FLOATS)
    return {"o": rec[:, 0:3].copy(), "d": rec[:, 3:6].copy(), "viewdir": rec[:, 6:9].copy(),
            "radius": rec[:, 9].copy(), "near": rec[:, 10].copy(), "far": rec[:, 11].copy(),
            "lossmult": rec[:, 12].copy(), "pix": rec[:, 13:16].copy()}
