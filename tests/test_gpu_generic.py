"""GPU parity of the any-shape fp32 network path (generic.hip) vs the fp64 oracle.

The reference's network is configurable (MLP.cs:64-86: depth, width, skip, the view branch's depth and
width, PE degrees); BASELINE configs[0] uses a 4x128 net.  Networks other than the fused kernels' 8x256
run layer by layer on MFMA GEMMs (accelerated.cpp gen_forward / gen_backward).  Same contract as
test_gpu_step.py: t bit-exact, outputs / integrator adjoint within 1e-5 with the oracle's own ReLU
decisions, the 2L gradient tensors within 1e-5 with the GPU's decisions adopted.
"""
import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-5

# (D, W, Dc, Wc, skip, min_deg, max_deg, deg_view)
SPECS = {
    "configs0_4x128": (4, 128, 1, 128, 4, 0, 16, 4),
    # widths off the 64-wide tiles, three condition layers, a skip every second layer, other PE degrees
    "odd_5x96_3x40": (5, 96, 3, 40, 2, 2, 10, 2),
    # skip into every layer, one-degree view PE
    "tiny_2x32_skip1": (2, 32, 1, 16, 1, 0, 4, 1),
    # deeper than the reference, two skips, no view PE harmonics
    "deep_10x64": (10, 64, 2, 32, 3, 0, 12, 0),
}


def _cfg(spec):
    D, W, Dc, Wc, skip, lo, hi, dv = spec
    return dict(net_depth=D, net_width=W, net_depth_condition=Dc, net_width_condition=Wc, skip_layer=skip,
                min_deg_point=lo, max_deg_point=hi, deg_view=dv)


def _ospec(oracle, spec):
    D, W, Dc, Wc, skip, lo, hi, dv = spec
    return oracle.Spec(D=D, W=W, Dc=Dc, Wc=Wc, skip=skip, min_deg=lo, max_deg=hi, deg_view=dv)


def _run(model, r, dev):
    import torch

    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in r.items()}
    n = r["o"].shape[0]
    msum = float(np.sum(r["lossmult"], dtype=np.float32))
    return model.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"],
                                     msum)


def _check(gpu, oracle, spec, kind, n, samples, lindisp=0, ray_shape=0, nthreads=16, lossmult=None, heads=None):
    import torch
    import nof
    from nof import synth

    seed, step, ray_base = 0x77, 2, 40
    opts = dict(lindisp=lindisp, ray_shape=ray_shape, **(heads or {}))
    model = nof.AcceleratedMipNeRF(seed=seed, max_rays=n, num_samples=samples, num_levels=len(samples), precision=0,
                                   **opts, **_cfg(spec))
    model.set_rng(seed, step, ray_base)
    sp = _ospec(oracle, spec)
    sizes = oracle.layer_sizes(sp)
    assert model.GetLayerSizes() == list(sizes)
    r = synth.blender_rays(n, seed=23) if kind == "blender" else synth.llff_rays(n, seed=23)
    if lossmult is not None:
        r["lossmult"] = np.resize(np.asarray(lossmult, np.float32), n)
    grads = _run(model, r, gpu)
    torch.cuda.synchronize()
    assert len(grads) == len(sizes)
    lv = [model.level_numpy(l) for l in range(len(samples))]
    pptr, P = model.mlp.flat_params()
    assert P == int(np.sum(sizes))
    params = nof.to_numpy(pptr, (P,))
    gptr, _ = model.mlp.flat_grads()
    G = nof.to_numpy(gptr, (P,))
    assert grads[0] == gptr

    t0 = oracle.sample_stratified(r["near"], r["far"], samples[0], True, seed, step, 0, ray_base, lindisp=bool(lindisp))
    assert np.array_equal(lv[0]["t"], t0)
    tov = {}
    for l in range(1, len(samples)):
        tl, _ = oracle.sample_pdf(lv[l - 1]["t"], lv[l - 1]["weights"], samples[l], 0.01, True, seed, step, l, ray_base)
        assert np.array_equal(lv[l]["t"], tl)
        tov[l] = lv[l]["t"]

    if lossmult is not None:  # masked rays: exactly zero output gradients
        for l in range(len(samples)):
            assert not np.any(lv[l]["density_grad"][r["lossmult"] == 0])
            assert not np.any(lv[l]["rgb_grad"][r["lossmult"] == 0])
    masks = {l: model.mlp.relu_masks(l).reshape(n, samples[l], -1) for l in range(len(samples))}
    kw = dict(samples=samples, seed=seed, step_idx=step, ray_base=ray_base, t_override=tov, nthreads=nthreads, **opts)
    ref = oracle.step(sp, params, r, relu_mask=masks, want=("grads",), **kw)
    free = oracle.step(sp, params, r, want=("sigma", "rgb", "w", "C", "dsigma", "drgb"), **kw)
    for l in range(len(samples)):
        for key, fk in (("density", "sigma"), ("rgb", "rgb"), ("weights", "w"), ("comp_rgb", "C"),
                        ("density_grad", "dsigma"), ("rgb_grad", "drgb")):
            e = rel_l2(lv[l][key], free[fk][l])
            assert e < TOL, f"{key} level {l}: rel L2 {e:.3g}"
    off, errs = 0, []
    for i, s in enumerate(sizes):
        e = rel_l2(G[off:off + s], ref["grads"][off:off + s])
        errs.append(e)
        assert e < TOL, f"gradient tensor {i} (size {s}): rel L2 {e:.3g}"
        off += s
    print(f"{spec}: gradient rel L2 max {max(errs):.2e} median {np.median(errs):.2e}")
    assert abs(model.loss() - free["loss"]) <= TOL * abs(free["loss"])
    model.close()


@pytest.mark.parametrize("name", list(SPECS))
def test_generic_step_parity(gpu, oracle, name):
    _check(gpu, oracle, SPECS[name], "blender", 8, (64, 128))


def test_generic_step_parity_llff_options(gpu, oracle):
    """NDC forward-facing rays, LinDisp sampling, cylinders and non-default heads (DensityBias / RgbPadding,
    MipNerfModel.cs:20,22) through the any-shape path."""
    _check(gpu, oracle, SPECS["odd_5x96_3x40"], "llff", 4, (64, 64), lindisp=1, ray_shape=1,
           heads=dict(density_bias=0.25, rgb_padding=0.01))


def test_generic_single_and_three_levels(gpu, oracle):
    _check(gpu, oracle, SPECS["configs0_4x128"], "blender", 6, (64,))
    _check(gpu, oracle, SPECS["tiny_2x32_skip1"], "blender", 4, (64, 64, 128))


# the edge cases of test_gpu_edges.py on the any-shape path: one ray, one ray at 512 + 512 samples, the fine
# level smaller than the coarse one, masked rays (lossmult = 0)
@pytest.mark.parametrize("n,samples,lossmult", [(1, (64, 64), None), (1, (512, 512), None), (5, (128, 64), None),
                                                (12, (64, 128), [1.0, 0.0, 2.0, 0.0])])
def test_generic_edges(gpu, oracle, n, samples, lossmult):
    _check(gpu, oracle, SPECS["odd_5x96_3x40"], "blender", n, samples, lossmult=lossmult)


def test_generic_configs0_fullsize(gpu, oracle):
    """BASELINE configs[0] at its size: 4096 rays x 64 (+64 resampled) samples, 4x128 MLP."""
    _check(gpu, oracle, SPECS["configs0_4x128"], "blender", 4096, (64, 64), nthreads=16)


def test_generic_per_level_and_deterministic(gpu):
    """get_gradient per level (MLPcpp:256-321: level 0 overwrites, level 1 accumulates) == the step's
    gradient, and two runs are bitwise equal (ordered split-K sums, no atomics)."""
    import torch
    import nof
    from nof import synth

    n = 32
    r = synth.blender_rays(n, seed=3)
    outs = []
    for _ in range(2):
        m = nof.AcceleratedMipNeRF(seed=4, max_rays=n, num_samples=(64, 128), **_cfg(SPECS["odd_5x96_3x40"]))
        _run(m, r, gpu)
        torch.cuda.synchronize()
        gp, P = m.mlp.flat_grads()
        outs.append(nof.to_numpy(gp, (P,)).copy())
        views = [m.level_view(l) for l in range(2)]
        for l in range(2):
            m.mlp.get_gradient(views[l]["rgb_grad"][0], views[l]["density_grad"][0], l)
        torch.cuda.synchronize()
        assert np.array_equal(nof.to_numpy(gp, (P,)), outs[-1])
        m.close()
    assert np.array_equal(outs[0], outs[1])


def test_generic_adam_training_lowers_loss(gpu):
    """A few steps of the training loop on the 4x128 net: Adam over the 2L-tensor arena, loss decreases."""
    import torch
    import nof
    from nof import synth

    n = 256
    r = synth.blender_rays(n, seed=8)
    m = nof.AcceleratedMipNeRF(seed=1, max_rays=n, num_samples=(64, 64), **_cfg(SPECS["configs0_4x128"]))
    adam = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)
    losses = []
    for s in range(30):
        m.set_rng(5, s, 0)
        g = _run(m, r, gpu)
        losses.append(m.loss())
        adam.step(m.mlp.allParams, g, 5e-3)
    torch.cuda.synchronize()
    assert np.all(np.isfinite(losses))
    assert losses[-1] < 0.7 * losses[0], losses
    adam.close()
    m.close()


def test_generic_matches_golden_fixture(gpu):
    """The any-shape path against the committed fixture of the INDEPENDENT restatement for configs[0]'s
    network (tests/golden/small_4x128.npz: tests/torch_ref.py fp64 autograd, 6 rays x 64+64, 4x128), not
    through the oracle: the GPU's Glorot init reproduces the fixture's checksum, level-0 t bit-exact,
    level-1 t within rounding, weights / composite / loss and the FULL gradient arena within 1e-5 (no ReLU
    decisions adopted: the fixture's fp64 z > 0 decide)."""
    import os
    import torch
    import nof
    from golden.make_golden import CASES

    c = CASES["small_4x128"]
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "small_4x128.npz"))
    rays = {k: g["ray_" + k] for k in ("o", "d", "radius", "near", "far", "lossmult", "pix")}
    n = rays["o"].shape[0]
    net = c["net"]
    model = nof.AcceleratedMipNeRF(seed=c["param_seed"], max_rays=n, num_samples=c["samples"], precision=0,
                                   **_cfg((net["D"], net["W"], net["Dc"], net["Wc"], 4, 0, 16, 4)))
    pptr, P = model.mlp.flat_params()
    params = nof.to_numpy(pptr, (P,)).copy()
    assert float(params.astype(np.float64).sum()) == float(g["param_checksum"]), "Glorot init differs from the fixture"
    model.set_rng(c["seed"], c["step"], c["ray_base"])
    _run(model, rays, gpu)
    torch.cuda.synchronize()
    lv = [model.level_numpy(l) for l in range(2)]
    assert np.array_equal(lv[0]["t"], g["t0"])
    assert np.allclose(lv[1]["t"], g["t1"], rtol=4e-7, atol=0)
    for l in range(2):
        assert rel_l2(lv[l]["weights"], g[f"w{l}"]) < TOL, f"weights level {l}"
        assert rel_l2(lv[l]["comp_rgb"], g[f"C{l}"]) < TOL, f"comp_rgb level {l}"
    assert abs(model.loss() - float(g["loss"])) <= TOL * abs(float(g["loss"]))
    G = nof.to_numpy(model.mlp.flat_grads()[0], (P,))
    sizes = model.GetLayerSizes()
    for i, (a, b) in enumerate(zip(np.split(G, np.cumsum(sizes)[:-1]), np.split(g["grads"], np.cumsum(sizes)[:-1]))):
        e = rel_l2(a, b)
        assert e < TOL, f"gradient tensor {i}: rel L2 {e:.3g}"
    model.close()


def test_generic_render_and_checkpoint(gpu, tmp_path):
    """render_device on an any-shape network == the training step's forward bitwise on the same Philox
    state; a checkpoint of the 2L-tensor arena + Adam state round-trips into a fresh model exactly."""
    import torch
    import nof
    from nof import synth

    n, samples = 40, (64, 128)
    r = synth.blender_rays(n, seed=31)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(gpu) for k, v in r.items()}
    cfg = _cfg(SPECS["odd_5x96_3x40"])
    m = nof.AcceleratedMipNeRF(seed=2, max_rays=n, num_samples=samples, **cfg)
    m.set_rng(0xABC, 4, 100)
    lv = m.render_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], randomized=True)
    torch.cuda.synchronize()
    out = [nof.to_numpy(*L["comp_rgb"]) for L in lv]
    m.set_rng(0xABC, 4, 100)
    g = _run(m, r, gpu)
    adam = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)
    adam.step(m.mlp.allParams, g, 1e-3)
    torch.cuda.synchronize()
    for l in range(2):
        assert np.array_equal(m.level_numpy(l)["comp_rgb"], out[l]), f"level {l}"
    path = str(tmp_path / "generic.ckpt")
    nof.save_checkpoint(path, m, adam)
    m2 = nof.AcceleratedMipNeRF(seed=99, max_rays=n, num_samples=samples, **cfg)
    adam2 = nof.AcceleratedAdamOptimizer(m2.GetLayerSizes(), m2.config)
    nof.load_checkpoint(path, m2, adam2)
    torch.cuda.synchronize()
    p1, P = m.mlp.flat_params()
    p2, _ = m2.mlp.flat_params()
    assert np.array_equal(nof.to_numpy(p1, (P,)), nof.to_numpy(p2, (P,)))
    assert adam2.iteration == 1 and m2.get_rng() == m.get_rng()
    ref = nof.AcceleratedMipNeRF(seed=99, max_rays=n, num_samples=samples, **_cfg(SPECS["tiny_2x32_skip1"]))
    with pytest.raises(nof.NofError):  # a different network's layout is refused
        nof.load_checkpoint(path, ref, nof.AcceleratedAdamOptimizer(ref.GetLayerSizes(), ref.config))
    for o in (adam, adam2):
        o.close()
    for o in (m, m2, ref):
        o.close()


def test_generic_native_and_python_drivers(gpu, tmp_path):
    """BASELINE configs[0] through both training drivers: bin/nof_train (the C ABI alone) and
    `python -m nof.train`, --net-depth 4 --net-width 128 --samples 64 64: both run, and the native driver's
    parameter dump is the finite 4x128 arena."""
    import os
    import subprocess
    import sys

    from nof import synth

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "nerf-or-nothing_amd", "bin", "nof_train")
    path = str(tmp_path / "rays.bin")
    synth.pack_records(synth.blender_rays(4096, seed=4)).tofile(path)
    dump = str(tmp_path / "params.bin")
    cmd = [exe, "--records", path, "--batch", "512", "--steps", "4", "--print-every", "2", "--seed", "77",
           "--net-depth", "4", "--net-width", "128", "--samples", "64,64", "--dump-params", dump,
           "--lindisp", "--cylinder", "--density-bias", "-0.5", "--rgb-padding", "0.002"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    P = np.fromfile(dump, np.float32)
    D, W, pos, dirs = 4, 128, 96, 27
    expect = pos * W + (D - 1) * W * W + W + 128 * (W + dirs) + 3 * 128 + (D * W + 1 + 128 + 3)
    assert P.size == expect and np.all(np.isfinite(P))
    env = dict(os.environ, PYTHONPATH=os.path.join(root, "nerf-or-nothing_amd"))
    q = subprocess.run([sys.executable, "-m", "nof.train", "--records", path, "--batch", "512", "--steps", "4",
                        "--print-every", "2", "--net-depth", "4", "--net-width", "128", "--samples", "64", "64",
                        "--lindisp", "--cylinder", "--density-bias", "-0.5", "--rgb-padding", "0.002"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert q.returncode == 0, q.stderr[-2000:]
    assert "rays/s" in q.stdout


def test_generic_encoded_api_path(gpu, oracle):
    """AcceleratedMLP.get_output / get_gradient (MLPcpp:214-321) on an any-shape network with encodings the
    caller computed (the oracle's, rounded to fp32) and FREED before get_gradient (the library keeps its own
    copy): density / rgb and the level's gradient match the fused step's level-0 results within 1e-5."""
    import torch
    import nof
    from nof import synth

    spec = SPECS["odd_5x96_3x40"]
    n, samples = 16, (64, 64)
    r = synth.blender_rays(n, seed=41)
    a = nof.AcceleratedMipNeRF(seed=6, max_rays=n, num_samples=samples, **_cfg(spec))
    b = nof.AcceleratedMipNeRF(seed=6, max_rays=n, num_samples=samples, **_cfg(spec))
    a.set_rng(9, 1, 0)
    _run(a, r, gpu)
    torch.cuda.synchronize()
    v0 = a.level_numpy(0)
    views = a.level_view(0)
    P = a.mlp.flat_grads()[1]
    a.mlp.get_gradient(views["rgb_grad"][0], views["density_grad"][0], 0)  # level 0 alone (overwrites)
    torch.cuda.synchronize()
    g_a = nof.to_numpy(a.mlp.flat_grads()[0], (P,)).copy()
    sp = _ospec(oracle, spec)
    mean, cov = oracle.cast(v0["t"], r["o"], r["d"], r["radius"])
    ep = torch.from_numpy(oracle.encode(sp, mean, cov).reshape(n * samples[0], -1).astype(np.float32)).to(gpu)
    ed = torch.from_numpy(oracle.dir_pe(sp, r["d"]).astype(np.float32)).to(gpu)
    dptr, rptr = b.mlp.get_output(ep, ed, 0, n, samples[0])
    torch.cuda.synchronize()
    assert rel_l2(nof.to_numpy(dptr, (n, samples[0])), v0["density"]) < TOL
    assert rel_l2(nof.to_numpy(rptr, (n, samples[0], 3)), v0["rgb"]) < TOL
    ep.fill_(float("nan"))  # the caller's buffers are gone before the backward
    ed.fill_(float("nan"))
    del ep, ed
    dg = torch.from_numpy(v0["density_grad"]).to(gpu)
    cg = torch.from_numpy(v0["rgb_grad"]).to(gpu)
    b.mlp.get_gradient(cg, dg, 0)
    torch.cuda.synchronize()
    g_b = nof.to_numpy(b.mlp.flat_grads()[0], (P,))
    assert np.all(np.isfinite(g_b))
    sizes = b.GetLayerSizes()
    for i, (x, y) in enumerate(zip(np.split(g_b, np.cumsum(sizes)[:-1]), np.split(g_a, np.cumsum(sizes)[:-1]))):
        assert rel_l2(x, y) < TOL, f"gradient tensor {i}"
    a.close()
    b.close()


def test_generic_get_output_refuses_more_rays_than_max_rays(gpu):
    """a call with fewer samples per ray than the level was built for fits the level's
    sample capacity with more rays than max_rays, but the per-ray buffers (view encodings, the view-layer
    gradient's ray sums) hold max_rays rays: refused with a status, and the object stays usable."""
    import torch
    import nof

    n, samples = 8, (64, 64)
    m = nof.AcceleratedMipNeRF(seed=6, max_rays=n, num_samples=samples, **_cfg(SPECS["odd_5x96_3x40"]))
    P, V = 2 * 3 * (10 - 2), 3 + 3 * 2 * 2  # IPE of degrees 2..9, view PE of degree 2 (the spec above)
    big = 2 * n  # 2n rays x 32 samples = the level's n x 64 capacity
    ep = torch.zeros(big * 32, P, device=gpu)
    ed = torch.zeros(big, V, device=gpu)
    with pytest.raises(nof.NofError):
        m.mlp.get_output(ep, ed, 0, big, 32)
    dptr, _ = m.mlp.get_output(ep[: n * 32], ed[:n], 0, n, 32)  # within max_rays: accepted
    torch.cuda.synchronize()
    assert np.all(np.isfinite(nof.to_numpy(dptr, (n, 32))))
    m.close()


def test_generic_more_than_65535_row_tiles(gpu):
    """8192 rays x 512 + 512 samples: 4.19 M samples per level = 65 536 GEMM row tiles, past a launch grid's
    y limit (the tiles are linear in x).  The step equals its two accumulated 4096-ray halves (global ray
    ids, the global loss-multiplier sum) within 1e-5."""
    import torch
    import nof
    from nof import synth

    n, samples = 8192, (512, 512)
    cfg = _cfg(SPECS["tiny_2x32_skip1"])
    r = synth.blender_rays(n, seed=12)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(gpu) for k, v in r.items()}
    msum = float(n)
    m = nof.AcceleratedMipNeRF(seed=3, max_rays=n, num_samples=samples, **cfg)
    m.set_rng(5, 1, 0)
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], msum)
    torch.cuda.synchronize()
    gp, P = m.mlp.flat_grads()
    g_full = nof.to_numpy(gp, (P,)).copy()
    assert np.all(np.isfinite(g_full)) and np.any(g_full != 0)
    m.close()
    h = n // 2
    m = nof.AcceleratedMipNeRF(seed=3, max_rays=h, num_samples=samples, **cfg)
    for i in range(2):
        sl = slice(i * h, (i + 1) * h)
        m.set_rng(5, 1, i * h)
        m.get_gradient_device(h, d["o"][sl], d["d"][sl], d["radius"][sl], d["near"][sl], d["far"][sl],
                              d["lossmult"][sl], d["pix"][sl], msum, accumulate=i > 0, publish=i == 1)
    torch.cuda.synchronize()
    g_acc = nof.to_numpy(m.mlp.flat_grads()[0], (P,))
    assert rel_l2(g_acc, g_full) < TOL
    m.close()
