"""CPU tests of the oracle: pinned by Random123 KAT vectors, golden fixtures from the independent
torch/numpy restatement (tests/golden), finite differences and hand-computed known answers."""
import os

import numpy as np
import pytest

import torch_ref as TR
from conftest import rel_l2

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Random123 kat_vectors: philox4x32 10 rounds (counter, key -> output)
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_philox_kat(oracle, ctr, key, out):
    assert tuple(int(x) for x in oracle.philox4x32_10(ctr, key)) == out
    got = TR.philox(*[np.array([c], np.uint32) for c in ctr], key[0], key[1])
    assert tuple(int(g[0]) for g in got) == out


def test_uniform_streams_agree(oracle):
    u = TR.uniforms(0x1234_5678_9ABC, 7, 1, 2, np.arange(100, 110), 33)
    ref = np.array([[oracle.uniform(0x1234_5678_9ABC, 7, 1, 2, r, k) for k in range(33)] for r in range(100, 110)],
                   np.float32)
    assert np.array_equal(u, ref)
    assert u.min() >= 0.0 and u.max() < 1.0


def _spec(oracle, net):
    return oracle.Spec(D=net["D"], W=net["W"], Dc=net["Dc"], Wc=net["Wc"])


@pytest.mark.parametrize("name", ["small_4x128", "ref_8x256"])
def test_oracle_matches_golden(oracle, name):
    from golden.make_golden import CASES

    c = CASES[name]
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = _spec(oracle, c["net"])
    net = TR.Net(**c["net"])
    P = TR.glorot(net, c["param_seed"])
    Po = oracle.glorot_init(spec, c["param_seed"])
    assert np.array_equal(P, Po), "oracle Glorot init != restatement"
    assert float(P.astype(np.float64).sum()) == float(g["param_checksum"])
    rays = {k: g["ray_" + k] for k in ("o", "d", "radius", "near", "far", "lossmult", "pix")}
    out = oracle.step(spec, P, rays, samples=c["samples"], seed=c["seed"], step_idx=c["step"],
                      ray_base=c["ray_base"], nthreads=4)
    for l in range(len(c["samples"])):
        assert np.array_equal(out["t"][l], g[f"t{l}"]), f"t level {l} not bit-exact"
        assert rel_l2(out["w"][l], g[f"w{l}"]) < 1e-12
        assert rel_l2(out["C"][l], g[f"C{l}"]) < 1e-12
    assert abs(out["loss"] - float(g["loss"])) < 1e-12 * abs(float(g["loss"]))
    G = out["grads"]
    if "grads" in g:
        assert rel_l2(G, g["grads"]) < 1e-10
    else:
        assert np.allclose(G[g["grad_idx"]], g["grad_vals"], rtol=1e-9, atol=1e-15)
    sizes = oracle.layer_sizes(spec)
    norms = np.array([np.linalg.norm(x) for x in np.split(G, np.cumsum(sizes)[:-1])])
    assert np.allclose(norms, g["grad_norms"], rtol=1e-10)


def test_resample_indices_match_brute_force(oracle):
    rng = np.random.default_rng(0)
    n, S = 16, 64
    near, far = np.full(n, 2, np.float32), np.full(n, 6, np.float32)
    t = oracle.sample_stratified(near, far, S, True, 1, 0, 0, 0)
    w = (rng.random((n, S)) ** 4).astype(np.float32)
    w[3] = 0.0
    t1, idx = oracle.sample_pdf(t, w, S, 0.01, True, 1, 0, 1, 0)
    u_raw = TR.uniforms(1, 0, 1, 2, np.arange(n), S + 1)
    t2, idx2 = TR.resample(t, w, S, 0.01, u_raw)
    assert np.array_equal(idx, idx2) and np.array_equal(t1, t2)
    assert np.all(np.diff(t1, axis=1) >= 0), "resampled t must be sorted"
    assert np.all(t1 >= t[:, :1]) and np.all(t1 <= t[:, -1:])
    assert idx.min() >= 0 and idx.max() <= S - 1


def test_stratified_deterministic_grid(oracle):
    t = oracle.sample_stratified(np.array([2.0], np.float32), np.array([6.0], np.float32), 8, False)
    assert np.allclose(t[0], np.linspace(2, 6, 9), atol=1e-6)
    tr = oracle.sample_stratified(np.array([2.0], np.float32), np.array([6.0], np.float32), 8, True, 3)
    lin = np.linspace(2, 6, 9)
    mids = 0.5 * (lin[1:] + lin[:-1])
    lower, upper = np.r_[lin[0], mids], np.r_[mids, lin[-1]]
    assert np.all(tr[0] >= lower - 1e-6) and np.all(tr[0] <= upper + 1e-6)


def test_render_known_answers(oracle):
    S = 4
    t = np.array([[2.0, 2.5, 3.0, 3.5, 4.0]], np.float32)
    d = np.array([[0.0, 0.0, -2.0]], np.float32)
    rgb = np.full((1, S, 3), 0.25)
    C, w = oracle.render(np.zeros((1, S)), rgb, t, d, white=True)      # alpha = 0 -> white background
    assert np.allclose(C, 1.0) and np.allclose(w, 0.0)
    sig = np.array([[0.7, 0.0, 0.0, 0.0]])
    C, w = oracle.render(sig, rgb, t, d, white=True)                   # one opaque-ish sample
    a = 1 - np.exp(-0.7 * 0.5 * 2.0)
    assert np.allclose(w[0, 0], a) and np.allclose(C, a * 0.25 + (1 - a))
    C, w = oracle.render(sig, rgb, t, d, white=False)
    assert np.allclose(C, a * 0.25)


def test_render_gradient_finite_difference(oracle):
    rng = np.random.default_rng(1)
    n, S = 3, 16
    t = np.sort(rng.random((n, S + 1)).astype(np.float32) * 4 + 2, axis=1)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    sig = rng.random((n, S)) * 3
    rgb = rng.random((n, S, 3))
    g = rng.standard_normal((n, 3))
    ds, dc = oracle.render_grad(g, sig, rgb, t, d, True)
    f = lambda s, c: float(np.sum(g * oracle.render(s, c, t, d, True)[0]))
    h = 1e-6
    for (r, k) in [(0, 0), (1, 7), (2, 15)]:
        e = np.zeros_like(sig); e[r, k] = h
        assert abs((f(sig + e, rgb) - f(sig - e, rgb)) / (2 * h) - ds[r, k]) < 1e-6
        e = np.zeros_like(rgb); e[r, k, 1] = h
        assert abs((f(sig, rgb + e) - f(sig, rgb - e)) / (2 * h) - dc[r, k, 1]) < 1e-6


def test_mlp_backward_finite_difference(oracle):
    spec = oracle.Spec(D=5, W=8, Dc=2, Wc=6, skip=4, max_deg=2, deg_view=1)  # exercises skip + 2 cond layers
    rng = np.random.default_rng(2)
    P = (rng.standard_normal(oracle.param_count(spec)) * 0.5).astype(np.float32)
    m = 5
    enc = rng.standard_normal((m, spec.pos_in))
    dirs = rng.standard_normal((m, spec.dir_in))
    dzs, dzc = rng.standard_normal(m), rng.standard_normal((m, 3))
    G = oracle.mlp_backward(spec, P, enc, dirs, dzs, dzc)

    def L(Pv):
        zs, zc, _ = oracle.mlp_forward(spec, Pv.astype(np.float32), enc, dirs)
        return float(np.dot(zs, dzs) + np.sum(zc * dzc))

    idx = rng.choice(P.size, 40, replace=False)
    for i in idx:  # params are float32, so perturb by an exactly representable step
        h = np.float32(2.0 ** -10)
        Pp, Pm = P.copy(), P.copy()
        Pp[i] += h
        Pm[i] -= h
        num = (L(Pp) - L(Pm)) / (float(Pp[i]) - float(Pm[i]))
        assert abs(num - G[i]) < 1e-6 * max(1.0, abs(G[i])) + 1e-9, f"param {i}"


def test_ipe_zero_variance_is_positional_encoding(oracle):
    spec = oracle.Spec(max_deg=6)
    mean = np.array([[0.3, -1.2, 2.5]], np.float32)
    enc = oracle.encode(spec, mean, np.zeros_like(mean))[0]
    for f in range(6):
        y = mean[0].astype(np.float64) * 2 ** f
        assert np.allclose(enc[6 * f:6 * f + 3], np.sin(y), atol=1e-12)
        assert np.allclose(enc[6 * f + 3:6 * f + 6], np.cos(y), atol=1e-5)  # sin(fl32(y + pi/2)) ~ cos(y)


def test_adam_and_lr_formulas(oracle):
    rng = np.random.default_rng(3)
    p = rng.standard_normal(1000).astype(np.float32)
    g = rng.standard_normal(1000).astype(np.float32) * np.float32(1e-2)
    m = np.zeros(1000, np.float32)
    v = np.zeros(1000, np.float32)
    p0 = p.copy()
    oracle.adam_step(p, g, m, v, 1e-3, 1)
    # first step from zero moments: m_hat = g, v_hat = g^2, so p moves by lr * g / sqrt(g^2 + eps)
    g64 = g.astype(np.float64)
    assert np.allclose(p, p0 - 1e-3 * g64 / np.sqrt(g64 ** 2 + 1e-8), rtol=0, atol=1e-6)
    lr = oracle.lr_decay(1)
    ref = (0.01 + 0.99 * np.sin(0.5 * np.pi / 2500)) * np.exp(np.log(5e-4) * (1 - 1e-6) + np.log(5e-6) * 1e-6)
    assert abs(lr - ref) < 1e-9
    assert abs(oracle.lr_decay(1000000) - 5e-6) < 1e-10


@pytest.mark.parametrize("lindisp,ray_shape", [(1, 0), (0, 1), (1, 1)])
def test_ray_options_match_independent_restatement(oracle, lindisp, ray_shape):
    """LinDisp sampling (MipNerfModel.cs:14, MipHelpers.cs:618-620) and cylinders (MipNerfModel.cs:15,
    MipHelpers.cs:403-409): the oracle's t-values and Gaussians bit-exact, and its whole two-level step
    (fp64) within 1e-9, against the independent numpy / torch-autograd restatement (tests/torch_ref.py)."""
    from nof import synth

    n, samples, seed, step, base = 3, (16, 16), 0x77, 2, 40
    spec = oracle.Spec(D=4, W=32, skip=2)
    r = synth.blender_rays(n, seed=5)
    P = oracle.glorot_init(spec, 9)
    gids = np.arange(base, base + n)
    t_ref = TR.stratified(r["near"], r["far"], samples[0], TR.uniforms(seed, step, 0, 1, gids, samples[0] + 1),
                          bool(lindisp))
    t = oracle.sample_stratified(r["near"], r["far"], samples[0], True, seed, step, 0, base, lindisp=bool(lindisp))
    assert np.array_equal(t, t_ref), "stratified t"
    if lindisp:  # disparity-linear: the un-jittered grid's inverse is linear in s
        g = oracle.sample_stratified(r["near"], r["far"], samples[0], False, lindisp=True)
        inv = 1.0 / g.astype(np.float64)
        assert np.allclose(np.diff(inv, 2, axis=1), 0, atol=1e-5 * np.abs(inv).max())
    m, c = oracle.cast(t, r["o"], r["d"], r["radius"], ray_shape)
    m_ref, c_ref = TR.cast(t, r["o"], r["d"], r["radius"], bool(ray_shape))
    assert np.array_equal(m, m_ref) and np.array_equal(c, c_ref), "Gaussians"
    net = TR.Net(D=4, W=32, skip=2)
    ref = TR.step(P, r, samples=samples, seed=seed, step_idx=step, ray_base=base, net=net, lindisp=bool(lindisp),
                  cylinder=bool(ray_shape))
    got = oracle.step(spec, P, r, samples=samples, seed=seed, step_idx=step, ray_base=base, nthreads=1,
                      lindisp=bool(lindisp), ray_shape=ray_shape)
    for l in range(2):
        assert np.array_equal(got["t"][l], ref["t"][l]), f"t level {l}"
        assert np.allclose(got["w"][l], ref["w"][l], rtol=1e-9, atol=1e-12), f"weights level {l}"
    assert abs(got["loss"] - ref["loss"]) <= 1e-9 * abs(ref["loss"])
    e = np.linalg.norm(got["grads"] - ref["grads"]) / np.linalg.norm(ref["grads"])
    assert e < 1e-9, f"gradients rel L2 {e:.3g}"


@pytest.mark.parametrize("density_bias,rgb_padding", [(-1.0, 0.001), (0.5, 0.02), (-3.0, 0.0)])
def test_head_options_match_independent_restatement(oracle, density_bias, rgb_padding):
    """MipNerfModel.DensityBias / RgbPadding (MipNerfModel.cs:20,22; the heads MNcs:19-28,151-152,184-189)
    as settable step options: the oracle's fp64 step within 1e-9 of the torch-autograd restatement."""
    from nof import synth

    spec = oracle.Spec(D=4, W=32, skip=2)
    r = synth.blender_rays(3, seed=5)
    P = oracle.glorot_init(spec, 9)
    ref = TR.step(P, r, samples=(16, 16), seed=0x77, step_idx=2, ray_base=40, net=TR.Net(D=4, W=32, skip=2),
                  density_bias=density_bias, rgb_padding=rgb_padding)
    got = oracle.step(spec, P, r, samples=(16, 16), seed=0x77, step_idx=2, ray_base=40, nthreads=1,
                      density_bias=density_bias, rgb_padding=rgb_padding)
    assert abs(got["loss"] - ref["loss"]) <= 1e-9 * abs(ref["loss"])
    e = np.linalg.norm(got["grads"] - ref["grads"]) / np.linalg.norm(ref["grads"])
    assert e < 1e-9, f"gradients rel L2 {e:.3g}"
