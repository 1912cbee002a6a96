"""Independent restatement of the mip-NeRF step in numpy (fp32 geometry) + PyTorch fp64 autograd.

TEST INFRASTRUCTURE.  Written separately from oracle/oracle.cpp (vectorised, autograd
instead of a hand-written backward, its own numpy Philox) so the two can pin each other:
``tests/golden/make_golden.py`` freezes this module's outputs as fixtures and the CPU
suite checks the C++ oracle against them.  Reference citations as in oracle.cpp.
"""
from __future__ import annotations

import numpy as np
import torch

M0, M1, W0, W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 on uint32 numpy arrays."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint32).copy() for x in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    for _ in range(10):
        p0 = c0.astype(np.uint64) * M0
        p1 = c2.astype(np.uint64) * M1
        n0 = (p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0
        n1 = (p1 & MASK).astype(np.uint32)
        n2 = (p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1
        n3 = (p0 & MASK).astype(np.uint32)
        c0, c1, c2, c3 = n0, n1, n2, n3
        k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def uniforms(seed, step, level, stream, rays, count):
    """u[r, k] for global ray ids ``rays`` and k in [0, count)."""
    rays = np.asarray(rays, np.uint32)
    k = np.arange(count, dtype=np.uint32)
    R, K = np.meshgrid(rays, k, indexing="ij")
    c2 = np.uint32((level & 0xFFFF) | (stream << 16))
    outs = philox(K >> np.uint32(2), R, np.full_like(R, c2), np.full_like(R, step), seed & 0xFFFFFFFF, seed >> 32)
    sel = np.stack(outs, 0)[(K & np.uint32(3)).astype(np.int64), np.arange(R.shape[0])[:, None], np.arange(R.shape[1])[None, :]]
    return (sel >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


f32 = np.float32


def stratified(near, far, S, u, lindisp=False):
    """SampleAlongRay (MipHelpers.cs:611-631); lindisp: linear in disparity (MipHelpers.cs:618-620)"""
    tv = np.arange(S + 1, dtype=f32) / f32(S)
    if lindisp:
        lin = f32(1) / (f32(1) / near[:, None] * (f32(1) - tv)[None, :] + f32(1) / far[:, None] * tv[None, :])
    else:
        lin = near[:, None] * (f32(1) - tv)[None, :] + far[:, None] * tv[None, :]
    mids = f32(0.5) * (lin[:, :-1] + lin[:, 1:])
    lower = np.concatenate([lin[:, :1], mids], 1)
    upper = np.concatenate([mids, lin[:, -1:]], 1)
    return (lower + (upper - lower) * u).astype(f32)


def resample(t, w, S_out, padding, u_raw):
    n, B = w.shape
    wpad = np.concatenate([w[:, :1], w, w[:, -1:]], 1)
    wmax = np.maximum(wpad[:, :-1], wpad[:, 1:])
    wb = (f32(0.5) * (wmax[:, :-1] + wmax[:, 1:]) + f32(padding)).astype(f32)
    wsum = wb.astype(np.float64).sum(1).astype(f32)
    pad = np.maximum(f32(0), f32(1e-5) - wsum)
    wb = np.where(pad[:, None] > 0, wb + (pad / f32(B))[:, None], wb).astype(f32)
    wsum = np.where(pad > 0, wsum + pad, wsum).astype(f32)
    pdf = (wb / wsum[:, None]).astype(f32)
    run = np.cumsum(pdf[:, :-1], axis=1, dtype=f32)
    cdf = np.concatenate([np.zeros((n, 1), f32), np.minimum(f32(1), run), np.ones((n, 1), f32)], 1)
    ns = S_out + 1
    s1 = f32(1) / f32(ns)
    i = np.arange(ns, dtype=f32)[None, :]
    u = np.minimum(i * s1 + u_raw * (s1 - f32(1e-7)), f32(1) - f32(1e-7)).astype(f32)
    idx = np.stack([np.searchsorted(cdf[r], u[r], side="right") - 1 for r in range(n)])
    idx = np.clip(idx, 0, B - 1)
    g = lambda a, j: np.take_along_axis(a, j, 1)
    b0, b1, c0, c1 = g(t, idx), g(t, idx + 1), g(cdf, idx), g(cdf, idx + 1)
    den = (c1 - c0).astype(f32)
    with np.errstate(divide="ignore", invalid="ignore"):
        tt = np.where(den > 0, (u - c0) / den, f32(0)).astype(f32)
    tt = np.clip(tt, f32(0), f32(1))
    return (b0 + tt * (b1 - b0)).astype(f32), idx.astype(np.int32)


def cast(t, o, d, radius, cylinder=False):
    """CastRay (MipHelpers.cs:410-428): ConicalFrustumToGaussian (MipHelpers.cs:391-402) or, cylinder,
    CylinderToGaussian (MipHelpers.cs:403-409), lifted by LiftGaussian (MipHelpers.cs:367-379)"""
    t0, t1 = t[:, :-1], t[:, 1:]
    if cylinder:
        tmean = (t0 + t1) / f32(2)
        rvar = np.broadcast_to(radius[:, None] * radius[:, None] / f32(4), tmean.shape)
        tvar = (t1 - t0) * (t1 - t0) / f32(12)
    else:
        mu = (t0 + t1) / f32(2)
        hw = (t1 - t0) / f32(2)
        mu2, hw2 = mu * mu, hw * hw
        den = f32(3) * mu2 + hw2
        tmean = mu + (f32(2) * mu * hw2) / den
        tvar = hw2 / f32(3) - (f32(4) / f32(15)) * (hw2 * hw2 * (f32(12) * mu2 - hw2)) / (den * den)
        rvar = radius[:, None] * radius[:, None] * (mu2 / f32(4) + (f32(5) / f32(12)) * hw2 - (f32(4) / f32(15)) * (hw2 * hw2) / den)
    dms = np.maximum(f32(1e-10), (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    dd = d * d
    nul = f32(1) - dd / dms[:, None]
    mean = d[:, None, :] * tmean[..., None] + o[:, None, :]
    cov = tvar[..., None] * dd[:, None, :] + rvar[..., None] * nul[:, None, :]
    return mean.astype(f32), cov.astype(f32)


def ipe(mean, cov, min_deg=0, max_deg=16):
    feats = []
    half_pi = f32(3.14159274) * f32(0.5)
    for f in range(min_deg, max_deg):
        s = f32(1 << f)
        y = mean * s
        yv = cov * s * s
        damp = np.exp(-0.5 * yv.astype(np.float64))
        feats.append(damp * np.sin(y.astype(np.float64)))
        feats.append(damp * np.sin((y + half_pi).astype(np.float64)))
    return np.concatenate(feats, -1)


def dir_pe(d, deg):
    out = [d.astype(np.float64)]
    for f in range(deg):
        xb = (d * f32(1 << f)).astype(np.float64)
        out += [np.sin(xb), np.cos(xb)]
    return np.concatenate(out, -1)


class Net:
    """Parameter views over the flat arena [W0..W_{L-1}, b0..b_{L-1}] (MLPcpp:131-154)."""

    def __init__(self, D=8, W=256, Dc=1, Wc=128, skip=4, pos_in=96, dir_in=27):
        self.D, self.W, self.Dc, self.Wc, self.skip = D, W, Dc, Wc, skip
        outs, ins = [W], [pos_in]
        for l in range(1, D):
            outs.append(W)
            ins.append(W + (pos_in if l % skip == 0 else 0))
        outs.append(1); ins.append(W)
        outs.append(Wc); ins.append(W + dir_in)
        for _ in range(1, Dc):
            outs.append(Wc); ins.append(Wc)
        outs.append(3); ins.append(Wc)
        self.outs, self.ins = outs, ins
        self.L = len(outs)

    def views(self, P):
        Ws, bs, o = [], [], 0
        for l in range(self.L):
            n = self.outs[l] * self.ins[l]
            Ws.append(P[o:o + n].view(self.outs[l], self.ins[l])); o += n
        for l in range(self.L):
            bs.append(P[o:o + self.outs[l]]); o += self.outs[l]
        return Ws, bs

    def forward(self, P, enc, dirv):
        Ws, bs = self.views(P)
        h = enc
        for l in range(self.D):
            x = torch.cat([h, enc], -1) if (l % self.skip == 0 and l > 0) else h
            h = torch.relu(x @ Ws[l].T + bs[l])
        zs = (h @ Ws[self.D].T + bs[self.D])[..., 0]
        x = torch.cat([h, dirv], -1)
        for i in range(self.Dc):
            l = self.D + 1 + i
            x = torch.relu(x @ Ws[l].T + bs[l])
        zc = x @ Ws[-1].T + bs[-1]
        return zs, zc


def render(sigma, rgb, t, d, white=True):
    dl = torch.from_numpy(np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(f32)).double()
    delta = torch.from_numpy((t[:, 1:] - t[:, :-1]).astype(f32)).double()
    alpha = 1 - torch.exp(-sigma * delta * dl[:, None])
    trans = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1 - alpha[:, :-1]], 1), 1)
    w = alpha * trans
    C = (w[..., None] * rgb).sum(1)
    if white:
        C = C + (1 - w.sum(1))[:, None]
    return C, w


def step(P_np, rays, samples=(128, 128), seed=0, step_idx=0, ray_base=0, padding=0.01, coarse_mult=0.1,
         white=True, net=None, t_override=None, lindisp=False, cylinder=False, density_bias=-1.0, rgb_padding=0.001):
    """Full two-level step; returns dict with t, w, C per level, loss, grads (fp64 autograd)."""
    net = net or Net()
    n = rays["o"].shape[0]
    gids = np.arange(ray_base, ray_base + n)
    P = torch.tensor(P_np, dtype=torch.float64, requires_grad=True)
    o, d, rad = rays["o"], rays["d"], rays["radius"]
    dirv = torch.from_numpy(dir_pe(d, 4))
    msum = float(np.sum(rays["lossmult"], dtype=np.float32))
    pix = torch.from_numpy(rays["pix"]).double()
    lm = torch.from_numpy(rays["lossmult"]).double()
    res = {"t": [], "w": [], "C": [], "idx": []}
    loss = 0
    NL = len(samples)
    for lv, S in enumerate(samples):
        if lv == 0:
            t = stratified(rays["near"], rays["far"], S, uniforms(seed, step_idx, 0, 1, gids, S + 1), lindisp)
            idx = None
        elif t_override is not None and lv in t_override:
            t, idx = t_override[lv], None
        else:
            wprev = res["w"][-1].detach().numpy().astype(f32)
            t, idx = resample(res["t"][-1], wprev, S, padding, uniforms(seed, step_idx, lv, 2, gids, S + 1))
        mean, cov = cast(t, o, d, rad, cylinder)
        enc = torch.from_numpy(ipe(mean, cov))
        zs, zc = net.forward(P, enc, dirv[:, None, :].expand(n, S, dirv.shape[-1]))
        # MipNerfModel.DensityBias / RgbPadding (MNcs:20-22), the scale (1 + 2 pad) formed in fp32 as in C#
        pad = np.float32(rgb_padding)
        sigma = torch.nn.functional.softplus(zs + float(np.float32(density_bias)), beta=1, threshold=20)
        rgb = torch.sigmoid(zc) * float(np.float32(1) + np.float32(2) * pad) - float(pad)
        C, w = render(sigma, rgb, t, d, white)
        lam = float(np.float32(coarse_mult)) if lv < NL - 1 else 1.0
        loss = loss + lam * (lm[:, None] * (C - pix) ** 2).sum() / msum
        res["t"].append(t); res["w"].append(w); res["C"].append(C); res["idx"].append(idx)
    loss.backward()
    res["grads"] = P.grad.numpy()
    res["loss"] = float(loss.detach())
    res["w"] = [w.detach().numpy() for w in res["w"]]
    res["C"] = [C.detach().numpy() for C in res["C"]]
    return res


def glorot(net: Net, seed: int) -> np.ndarray:
    """C#-semantics Glorot init (MLPcs:78-85): W = sqrt(6/(in+out)) (2u - 1), b = 0; u from Philox
    (seed, step 0, level = layer, stream 3, ray = e >> 32, k = e)."""
    P = []
    for l in range(net.L):
        cnt = net.outs[l] * net.ins[l]
        e = np.arange(cnt, dtype=np.uint64)
        k = (e & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        c2 = np.uint32((l & 0xFFFF) | (3 << 16))
        outs = philox(k >> np.uint32(2), (e >> np.uint64(32)).astype(np.uint32), np.full(cnt, c2, np.uint32),
                      np.zeros(cnt, np.uint32), seed & 0xFFFFFFFF, seed >> 32)
        sel = np.stack(outs, 0)[(k & np.uint32(3)).astype(np.int64), np.arange(cnt)]
        u = (sel >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        g = np.sqrt(np.float32(6.0) / np.float32(net.ins[l] + net.outs[l])).astype(np.float32)
        P.append((g * (u * np.float32(2) - np.float32(1))).astype(np.float32))
    P += [np.zeros(o, np.float32) for o in net.outs]
    return np.concatenate(P)
