"""CPU oracle for device ray generation (TEST INFRASTRUCTURE ONLY — never imported by the product).

float32 numpy restatement, operation by operation in the C# evaluation order, of
  * Dataset.GenerateRays            ScratchNerf/Dataset.cs:111-176
  * LLFFDataset.GenerateRays        ScratchNerf/Dataset.cs:268-293
  * LLFFDataset.ConvertToNdc        ScratchNerf/Dataset.cs:295-308
  * LLFFDataset.RecenterPoses       ScratchNerf/Dataset.cs:309-319
  * Matrix3x3 * Vector3 / Matrix3x3 ScratchNerf/MipHelpers.cs:24-40
Vector3.Length is taken as sqrt((x*x + y*y) + z*z) (the .NET SIMD dot order is not pinned: parity
unpinned at that one rounding).  Output: BinDataset records [V*H*W, 16] (BinDataset.cs:40-49).
"""
import numpy as np

f32 = np.float32


def _len3(x, y, z):
    return np.sqrt((x * x + y * y) + z * z)


def pixel_dirs(P, xs, ys, w, h, focal):
    """cameraDirs then rotation * dir for pixel arrays xs, ys (Dataset.cs:118-141)."""
    cx = (xs.astype(f32) - f32(w) * f32(0.5) + f32(0.5)) / f32(focal)
    cy = -(ys.astype(f32) - f32(h) * f32(0.5) + f32(0.5)) / f32(focal)
    cz = np.full_like(cx, f32(-1.0))
    R = np.asarray(P[:9], f32)
    return [(R[3 * i] * cx + R[3 * i + 1] * cy) + R[3 * i + 2] * cz for i in range(3)]


def to_ndc(o, d, focal, w, h):
    nearp = f32(1.0)
    t = -(nearp + o[2]) / d[2]
    ox, oy, oz = o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]
    a = f32(2.0) * f32(focal) / f32(w)
    b = f32(2.0) * f32(focal) / f32(h)
    on = [-a * (ox / oz), -b * (oy / oz), f32(1.0) + f32(2.0) * nearp / oz]
    dn = [-a * (d[0] / d[2] - ox / oz), -b * (d[1] / d[2] - oy / oz), -f32(2.0) * nearp / oz]
    return on, dn


def generate(poses, w, h, focal, near, far, ndc=False, images=None):
    poses = np.asarray(poses, f32).reshape(-1, 12)
    V = poses.shape[0]
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    xs, ys = xs.ravel(), ys.ravel()
    out = np.zeros((V, h * w, 16), f32)
    for v in range(V):
        P = poses[v]
        d = pixel_dirs(P, xs, ys, w, h, focal)
        dl = _len3(*d)
        vd = [d[0] / dl, d[1] / dl, d[2] / dl]
        o = [np.full_like(d[0], P[9]), np.full_like(d[0], P[10]), np.full_like(d[0], P[11])]
        if not ndc:
            nx = np.where(xs < w - 1, xs + 1, xs)
            dn = pixel_dirs(P, nx, ys, w, h, focal)
            radius = _len3(d[0] - dn[0], d[1] - dn[1], d[2] - dn[2]) * f32(2.0) / np.sqrt(f32(12.0))
            dd = d
        else:
            on, dd = to_ndc(o, d, focal, w, h)

            def ndc_o(x2, y2):
                return to_ndc(o, pixel_dirs(P, x2, y2, w, h, focal), focal, w, h)[0]

            right, left = ndc_o(np.minimum(xs + 1, w - 1), ys), ndc_o(np.maximum(xs - 1, 0), ys)
            down, up = ndc_o(xs, np.minimum(ys + 1, h - 1)), ndc_o(xs, np.maximum(ys - 1, 0))
            lastx, lasty = xs >= w - 1, ys >= h - 1
            ax = [np.where(lastx, left[i], on[i]) for i in range(3)]
            bx = [np.where(lastx, on[i], right[i]) for i in range(3)]
            ay = [np.where(lasty, up[i], on[i]) for i in range(3)]
            by = [np.where(lasty, on[i], down[i]) for i in range(3)]
            dx = _len3(ax[0] - bx[0], ax[1] - bx[1], ax[2] - bx[2])
            dy = _len3(ay[0] - by[0], ay[1] - by[1], ay[2] - by[2])
            radius = np.sqrt(dx * dx + dy * dy) / np.sqrt(f32(12.0))
            o = on
        rec = out[v]
        rec[:, 0], rec[:, 1], rec[:, 2] = o
        rec[:, 3], rec[:, 4], rec[:, 5] = dd
        rec[:, 6], rec[:, 7], rec[:, 8] = vd
        rec[:, 9], rec[:, 10], rec[:, 11], rec[:, 12] = radius, near, far, 1.0
        if images is not None:
            rec[:, 13:16] = np.asarray(images[v], f32).reshape(-1, 3)
    return out.reshape(-1, 16)


def recenter_poses(poses):
    P = np.array(poses, f32).reshape(-1, 12).copy()
    V = P.shape[0]
    R, t = P[0, :9].copy(), P[0, 9:].copy()
    for i in range(1, V):
        R, t = R + P[i, :9], t + P[i, 9:]
    R, t = R / f32(V), t / f32(V)
    Ri = R.reshape(3, 3).T.ravel()
    ti = np.array([(-Ri[3 * r] * t[0] + -Ri[3 * r + 1] * t[1]) + -Ri[3 * r + 2] * t[2] for r in range(3)], f32)
    for i in range(V):
        Rp = P[i, :9].copy()
        u = np.array([(Rp[3 * r] * ti[0] + Rp[3 * r + 1] * ti[1]) + Rp[3 * r + 2] * ti[2] for r in range(3)], f32)
        P[i, 9:] = P[i, 9:] - u
        P[i, :9] = np.array([(Rp[3 * r] * Ri[c] + Rp[3 * r + 1] * Ri[3 + c]) + Rp[3 * r + 2] * Ri[6 + c]
                             for r in range(3) for c in range(3)], f32)
    return P
