"""GPU parity of the whole training step (AcceleratedMipNeRF.GetGradient) vs the fp64 oracle.

Level-1 t-values are resampled on the GPU from the GPU's level-0 weights; they are checked
bit-exactly against the oracle's resampler fed those same weights, and then injected into the
oracle step (t_override) so that every other tensor is compared on identical samples.
"""
import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-5
# per-tensor relative L2 bound per precision mode: fp32 and the bf16x3 split mode are
# fp32-accurate, and so is the fp16 (hi, lo) split in every contraction (F32_F16SPLIT); the f16x2 perf
# mode (one fp16 product per weight-gradient term) is bounded at 2e-3
TOLS = {0: 1e-5, 1: 1e-5, 2: 2e-3, 3: 1e-5, 4: 2e-3}


def _device_rays(r, dev):
    import torch

    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in r.items()}


def _run_gpu(model, r, dev, msum=None):
    d = _device_rays(r, dev)
    n = r["o"].shape[0]
    msum = float(np.sum(r["lossmult"], dtype=np.float32)) if msum is None else msum
    return model.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], msum)


# NOF_PRECISION_F32, _F32_SPLIT (both 1e-5), _F16X2 (perf mode, 2e-3), _F32_F16SPLIT (1e-5)
PRECISIONS = [0, 1, 2, 3, 4]


# blender = configs 2/3 shapes (64+128 = config 3); llff = config 5's NDC forward-facing rays at
# 256 samples per level (config 5 runs fp16 on MFMA: precision 2)
@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("kind,n,samples", [("blender", 16, (64, 64)), ("blender", 8, (128, 128)),
                                            ("blender", 6, (64, 128)), ("llff", 3, (256, 256))])
def test_step_parity(gpu, oracle, kind, n, samples, precision):
    _check_step(gpu, oracle, kind, n, samples, precision)


# the spec's non-default ray options (MipNerfModel.cs:14-15): LinDisp sampling (MH:618-620) and cylinders
# (CylinderToGaussian MH:403-409), through the fp32 / split / F16 forward kernels' fused prologues
@pytest.mark.parametrize("precision", [0, 1, 4])
@pytest.mark.parametrize("lindisp,ray_shape", [(1, 0), (0, 1), (1, 1)])
def test_step_parity_ray_options(gpu, oracle, lindisp, ray_shape, precision):
    _check_step(gpu, oracle, "blender", 8, (64, 128), precision, lindisp=lindisp, ray_shape=ray_shape)


# MipNerfModel.DensityBias / RgbPadding (MipNerfModel.cs:20,22) away from their defaults, every precision mode
@pytest.mark.parametrize("precision", PRECISIONS)
def test_step_parity_head_options(gpu, oracle, precision):
    _check_step(gpu, oracle, "blender", 8, (64, 128), precision, heads=dict(density_bias=0.5, rgb_padding=0.02))


def _check_step(gpu, oracle, kind, n, samples, precision, lindisp=0, ray_shape=0, heads=None):
    import torch
    import nof
    from nof import synth

    seed, step, ray_base = 0x1234, 3, 500
    opts = dict(lindisp=lindisp, ray_shape=ray_shape, **(heads or {}))
    model = nof.AcceleratedMipNeRF(seed=seed, max_rays=n, num_samples=samples, precision=precision, **opts)
    model.set_rng(seed, step, ray_base)
    r = synth.blender_rays(n, seed=11) if kind == "blender" else synth.llff_rays(n, seed=11)
    grads = _run_gpu(model, r, gpu)
    torch.cuda.synchronize()
    lv = [model.level_numpy(l) for l in range(len(samples))]
    pptr, P = model.mlp.flat_params()
    params = nof.to_numpy(pptr, (P,))
    gptr, _ = model.mlp.flat_grads()
    G = nof.to_numpy(gptr, (P,))
    assert grads[0] == gptr

    # level-0 samples: bit-exact; level-1 resampling: bit-exact given the GPU's level-0 weights
    t0 = oracle.sample_stratified(r["near"], r["far"], samples[0], True, seed, step, 0, ray_base, lindisp=bool(lindisp))
    assert np.array_equal(lv[0]["t"], t0)
    t1, _ = oracle.sample_pdf(lv[0]["t"], lv[0]["weights"], samples[1], 0.01, True, seed, step, 1, ray_base)
    assert np.array_equal(lv[1]["t"], t1)

    # For the MLP gradients the oracle adopts the GPU's ReLU decisions: a pre-activation at ~0 may round
    # to opposite signs in fp32 and fp64, which would shift every gradient below that unit (measure-zero tie).
    masks = {l: model.mlp.relu_masks(l).reshape(n, samples[l], -1) for l in range(len(samples))}
    ref = oracle.step(oracle.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=ray_base,
                      t_override={1: lv[1]["t"]}, relu_mask=masks, nthreads=16, **opts)
    # forward outputs and the integrator adjoint: the oracle's own ReLU decisions (no adoption)
    free = oracle.step(oracle.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=ray_base,
                       t_override={1: lv[1]["t"]}, nthreads=16, want=("sigma", "rgb", "w", "C", "dsigma", "drgb"),
                       **opts)
    tol = TOLS[precision]
    for l in range(len(samples)):
        assert rel_l2(lv[l]["density"], free["sigma"][l]) < tol, f"density level {l}"
        assert rel_l2(lv[l]["rgb"], free["rgb"][l]) < tol, f"rgb level {l}"
        assert rel_l2(lv[l]["weights"], free["w"][l]) < tol, f"weights level {l}"
        assert rel_l2(lv[l]["comp_rgb"], free["C"][l]) < tol, f"comp_rgb level {l}"
        assert rel_l2(lv[l]["density_grad"], free["dsigma"][l]) < tol, f"dsigma level {l}"
        assert rel_l2(lv[l]["rgb_grad"], free["drgb"][l]) < tol, f"drgb level {l}"
    sizes = oracle.layer_sizes(oracle.Spec())
    off = 0
    errs = []
    for i, s in enumerate(sizes):
        e = rel_l2(G[off:off + s], ref["grads"][off:off + s])
        errs.append(e)
        assert e < tol, f"gradient tensor {i}: rel L2 {e:.3g}"
        off += s
    print(f"precision {precision}: gradient rel L2 max {max(errs):.2e} median {np.median(errs):.2e}")
    assert abs(model.loss() - free["loss"]) <= tol * abs(free["loss"])
    model.close()


@pytest.mark.parametrize("precision", PRECISIONS)
def test_per_level_gradient_equals_two_level_launch(gpu, precision):
    """AcceleratedMLP.get_gradient called per level (MLPcpp:256-321: level 0, then level 1 accumulating)
    == the step's one two-level weight-gradient launch.  In the f16 modes each level's deltas carry their
    own power-of-two scale, which the reduce must undo per level (a per-level call unscaled
    level 1 with level 0's word)."""
    import torch
    import nof
    from nof import synth

    n = 48
    r = synth.blender_rays(n, seed=17)
    model = nof.AcceleratedMipNeRF(seed=9, max_rays=n, num_samples=(64, 128), precision=precision)
    model.set_rng(11, 2, 0)
    _run_gpu(model, r, gpu)
    torch.cuda.synchronize()
    P = model.mlp.flat_grads()[1]
    g_fused = nof.to_numpy(model.mlp.flat_grads()[0], (P,)).copy()
    views = [model.level_view(l) for l in range(2)]
    for l in range(2):
        model.mlp.get_gradient(views[l]["rgb_grad"][0], views[l]["density_grad"][0], l)
    torch.cuda.synchronize()
    g_levels = nof.to_numpy(model.mlp.flat_grads()[0], (P,))
    sizes = model.GetLayerSizes()
    off = 0
    for i, s in enumerate(sizes):  # the two schedules cut the split-K items differently: fp32 rounding only
        e = rel_l2(g_levels[off:off + s], g_fused[off:off + s])
        assert e < 1e-5, f"gradient tensor {i}: per-level calls vs the two-level launch rel L2 {e:.3g}"
        off += s
    model.close()


def test_callback_path_equals_fused(gpu):
    """GetGradient(host arrays + AcceleratedGradientCalculator callback) == fused device path, bitwise."""
    import torch
    import nof
    from nof import synth

    n = 32
    r = synth.blender_rays(n, seed=5)
    a = nof.AcceleratedMipNeRF(seed=7, max_rays=n)
    b = nof.AcceleratedMipNeRF(seed=7, max_rays=n)
    gc = nof.AcceleratedGradientCalculator(n, b.config)
    _run_gpu(a, r, gpu)
    seen = []

    def cb(comp, level, msum, lm):
        seen.append(level)
        return gc.get_output_gradient(comp, r["pix"], lm, msum, level)

    b.GetGradient(r["o"], r["d"], r["radius"], r["near"], r["far"], r["lossmult"], cb)
    torch.cuda.synchronize()
    assert seen == [0, 1]
    ga = nof.to_numpy(a.mlp.flat_grads()[0], (546948,))
    gb = nof.to_numpy(b.mlp.flat_grads()[0], (546948,))
    assert np.array_equal(ga, gb)
    out = nof.OutputRetriever.RetrieveOutput(b.level_view(1)["comp_rgb"][0], n)
    assert np.array_equal(out, a.level_numpy(1)["comp_rgb"])


def test_encoded_get_output_equals_fused(gpu):
    """AcceleratedMLP.get_output on cast+encode kernels == the fused frustum/IPE forward, bitwise."""
    import torch
    import nof
    from nof import synth

    n, S = 8, 128
    r = synth.blender_rays(n, seed=9)
    model = nof.AcceleratedMipNeRF(seed=3, max_rays=n)
    _run_gpu(model, r, gpu)
    torch.cuda.synchronize()
    v0 = model.level_numpy(0)
    dev = _device_rays(r, gpu)
    t = torch.from_numpy(v0["t"]).to(gpu)
    mean = torch.zeros((n, S, 3), device=gpu)
    cov = torch.zeros((n, S, 3), device=gpu)
    nof._lib.call("nof_kernel_cast", n, S, t.data_ptr(), dev["o"].data_ptr(), dev["d"].data_ptr(),
                  dev["radius"].data_ptr(), mean.data_ptr(), cov.data_ptr(), None)
    ep = torch.zeros((n * S, 96), device=gpu)
    ed = torch.zeros((n, 27), device=gpu)
    nof._lib.call("nof_kernel_encode", n, S, mean.data_ptr(), cov.data_ptr(), dev["d"].data_ptr(), ep.data_ptr(),
                  ed.data_ptr(), None)
    dptr, rptr = model.mlp.get_output(ep, ed, 0, n, S)
    torch.cuda.synchronize()
    assert np.array_equal(nof.to_numpy(dptr, (n, S)), v0["density"])
    assert np.array_equal(nof.to_numpy(rptr, (n, S, 3)), v0["rgb"])


@pytest.mark.parametrize("precision", PRECISIONS)
def test_gradients_deterministic(gpu, precision):
    import torch
    import nof
    from nof import synth

    n = 64
    r = synth.blender_rays(n, seed=2)
    outs = []
    for _ in range(2):
        m = nof.AcceleratedMipNeRF(seed=5, max_rays=n, precision=precision)
        _run_gpu(m, r, gpu)
        torch.cuda.synchronize()
        outs.append(nof.to_numpy(m.mlp.flat_grads()[0], (546948,)))
        m.close()
    assert np.array_equal(outs[0], outs[1])
