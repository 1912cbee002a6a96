"""GPU parity vs the fp64 oracle at BASELINE sizes (VERDICT r1 "what's weak" 1).

The small-case step parity (test_gpu_step.py) runs 3-16 rays; these cases run the shapes bench.py
times, so the many-block paths (tail-block clamping in the forward kernels, per-M weight-gradient
schedules, slab growth) are checked against the oracle, not only by self-consistency:

* config 2: 1024 rays x 128+128 samples, fp32 and the bf16x3 split mode (1e-5 per tensor);
* config 3: 1024 rays x 64+128 (1e-5);
* config 5 per-GPU shape: 512 LLFF rays x 256+256, the f16x2 perf mode (2e-3) and fp32 (1e-5);
* config 4: one full 8192-ray shard on the GPU (global ray ids, global loss-mult sum) — per-ray
  outputs of its last 1024 rays (the tail blocks) vs the oracle — and the gradient of a 1024-ray
  slice of it; test_gpu_scale.py shows the shard's gradient is the sum of its slices.

Forward outputs, the integrator adjoint and the loss are compared with the oracle's own fp64 ReLU
decisions; for the MLP gradients the oracle adopts the GPU's decisions (as in test_gpu_step.py) and
the number of adopted decisions that differ from its own z > 0 is bounded too.
"""
import os

import numpy as np
import pytest

from conftest import f16_grad_tol, rel_l2

pytestmark = pytest.mark.gpu
TOLS = {0: 1e-5, 1: 1e-5, 2: 2e-3, 3: 1e-5, 4: 2e-3}
# adopted ReLU decisions that differ from the fp64 oracle's own, as a fraction of all units (ties at
# z ~ 0; measured 5e-8 .. 1.3e-7 in all three modes, the f16x2 mode included)
FLIP_BOUND = {0: 1e-5, 1: 1e-5, 2: 1e-5, 3: 1e-5, 4: 5e-4}  # f16: fp16 pre-activations (2^-11)
NTHREADS = min(16, len(os.sched_getaffinity(0)))
PER_RAY = ("density", "rgb", "weights", "comp_rgb", "density_grad", "rgb_grad")
ORACLE_KEY = {"density": "sigma", "rgb": "rgb", "weights": "w", "comp_rgb": "C", "density_grad": "dsigma",
              "rgb_grad": "drgb"}


def _rays(kind, n, seed):
    from nof import synth

    return synth.blender_rays(n, seed=seed) if kind == "blender" else synth.llff_rays(n, seed=seed)


def _gpu_step(model, r, gpu, msum, lo=0, hi=None):
    import torch

    hi = r["o"].shape[0] if hi is None else hi
    d = {k: torch.from_numpy(np.ascontiguousarray(v[lo:hi])).to(gpu) for k, v in r.items()}
    model.get_gradient_device(hi - lo, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"],
                              msum)
    torch.cuda.synchronize()


def _check_t(oracle, lv, r, samples, seed, step, base, lindisp=0):
    t0 = oracle.sample_stratified(r["near"], r["far"], samples[0], True, seed, step, 0, base, lindisp=bool(lindisp))
    assert np.array_equal(lv[0]["t"], t0), "level-0 t not bit-exact"
    t1, _ = oracle.sample_pdf(lv[0]["t"], lv[0]["weights"], samples[1], 0.01, True, seed, step, 1, base)
    assert np.array_equal(lv[1]["t"], t1), "level-1 t not bit-exact (given the GPU's level-0 weights)"


def _compare_step(oracle, model, r, samples, seed, step, base, msum, precision, lindisp=0, ray_shape=0):
    """Everything of one GPU step vs the oracle on the same samples; returns (max grad rel, flip frac).

    The forward outputs and the integrator adjoint (density, rgb, weights, comp_rgb, dsigma, drgb, the
    loss) are compared with an oracle run that makes its OWN ReLU decisions (fp64 z > 0); only the MLP
    gradients use a second oracle run that adopts the GPU's decisions (a tie at z ~ 0 gates every
    gradient below that unit), with the number of adopted decisions that differ bounded."""
    import nof

    n = r["o"].shape[0]
    tol = TOLS[precision]
    opts = dict(lindisp=lindisp, ray_shape=ray_shape)
    lv = [model.level_numpy(l) for l in range(len(samples))]
    _check_t(oracle, lv, r, samples, seed, step, base, lindisp)
    pptr, P = model.mlp.flat_params()
    params = nof.to_numpy(pptr, (P,))
    G = nof.to_numpy(model.mlp.flat_grads()[0], (P,))
    free = oracle.step(oracle.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=base,
                       loss_mult_sum=msum, t_override={1: lv[1]["t"]}, nthreads=NTHREADS,
                       want=tuple(ORACLE_KEY.values()), **opts)
    for l in range(len(samples)):
        for k in PER_RAY:
            e = rel_l2(lv[l][k], free[ORACLE_KEY[k]][l])
            assert e < tol, f"{k} level {l} (oracle's own ReLU decisions): rel L2 {e:.3g}"
    assert abs(model.loss() - free["loss"]) <= tol * abs(free["loss"])
    del free
    masks = {l: model.mlp.relu_masks(l).reshape(n, samples[l], -1) for l in range(len(samples))}
    ref = oracle.step(oracle.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=base,
                      loss_mult_sum=msum, t_override={1: lv[1]["t"]}, relu_mask=masks, nthreads=NTHREADS,
                      want=("grads",), **opts)
    units = sum(n * s * masks[l].shape[-1] for l, s in enumerate(samples))
    flips = sum(ref["mask_flips"]) / units
    del masks
    errs = []
    off = 0
    for i, s in enumerate(oracle.layer_sizes(oracle.Spec())):
        e = rel_l2(G[off:off + s], ref["grads"][off:off + s])
        errs.append(e)
        assert e < tol, f"gradient tensor {i}: rel L2 {e:.3g}"
        off += s
    assert flips < FLIP_BOUND[precision], f"adopted ReLU decisions differ in {flips:.3g} of the units"
    print(f"n={n} samples={samples} precision={precision}: gradient rel L2 max {max(errs):.2e} "
          f"median {np.median(errs):.2e}; ReLU flips {sum(ref['mask_flips'])} ({flips:.2e} of units)")
    return max(errs), flips


@pytest.mark.parametrize("name,kind,n,samples,precision", [
    ("config2", "blender", 1024, (128, 128), 0),
    ("config2", "blender", 1024, (128, 128), 1),
    ("config2", "blender", 1024, (128, 128), 2),
    ("config2", "blender", 1024, (128, 128), 3),
    ("config3", "blender", 1024, (64, 128), 0),
    ("config3", "blender", 1024, (64, 128), 1),
    ("config3", "blender", 1024, (64, 128), 2),
    ("config3", "blender", 1024, (64, 128), 3),
    ("config5", "llff", 512, (256, 256), 2),
    ("config5", "llff", 512, (256, 256), 0),
    ("config5", "llff", 512, (256, 256), 3),
    ("config2", "blender", 1024, (128, 128), 4),
    ("config5", "llff", 512, (256, 256), 4),
])
def test_fullsize_step_parity(gpu, oracle, name, kind, n, samples, precision):
    _fullsize(gpu, oracle, name, kind, n, samples, precision)


@pytest.mark.parametrize("precision", [0, 4])
def test_fullsize_ray_options(gpu, oracle, precision):
    """config 2 with the spec's non-default ray options (MipNerfModel.cs:14-15): LinDisp sampling and
    cylindrical Gaussians, fp32 and F16"""
    _fullsize(gpu, oracle, "config2", "blender", 1024, (128, 128), precision, lindisp=1, ray_shape=1)


def _fullsize(gpu, oracle, name, kind, n, samples, precision, **opts):
    import nof

    seed, step, base = 0x5EED0000 + int(name[-1]), 5, 0
    r = _rays(kind, n, seed=21)
    msum = float(np.sum(r["lossmult"], dtype=np.float32))
    model = nof.AcceleratedMipNeRF(seed=31, max_rays=n, num_samples=samples, precision=precision, **opts)
    model.set_rng(seed, step, base)
    _gpu_step(model, r, gpu, msum)
    _compare_step(oracle, model, r, samples, seed, step, base, msum, precision, **opts)
    model.close()


@pytest.mark.parametrize("name,kind,n,samples", [
    ("config2", "blender", 1024, (128, 128)),
    ("config5", "llff", 512, (256, 256)),
])
def test_f16_gradients_mask_free(gpu, oracle, name, kind, n, samples):
    """All 22 F16 gradient tensors vs an fp64 oracle run that makes its own fp64 z > 0 decisions.  The F16
    pre-activations are rounded to fp16 before the ReLU, so a unit with |z| within fp16 rounding of 0 may
    gate the other way; no decision is adopted here, so the per-tensor bound (f16_grad_tol, conftest.py: W0 and
    b0 6e-3, every other tensor 2e-3) covers those flips as well; the whole arena within 2e-3."""
    import nof

    seed, step, base = 0x5EED0000 + int(name[-1]), 5, 0
    r = _rays(kind, n, seed=21)
    msum = float(np.sum(r["lossmult"], dtype=np.float32))
    model = nof.AcceleratedMipNeRF(seed=31, max_rays=n, num_samples=samples, precision=4)
    model.set_rng(seed, step, base)
    _gpu_step(model, r, gpu, msum)
    lv = [model.level_numpy(l) for l in range(len(samples))]
    pptr, P = model.mlp.flat_params()
    params = nof.to_numpy(pptr, (P,))
    G = nof.to_numpy(model.mlp.flat_grads()[0], (P,))
    ref = oracle.step(oracle.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=base,
                      loss_mult_sum=msum, t_override={1: lv[1]["t"]}, nthreads=NTHREADS, want=("grads",))
    errs, off = [], 0
    for s in oracle.layer_sizes(oracle.Spec()):
        errs.append(rel_l2(G[off:off + s], ref["grads"][off:off + s]))
        off += s
    whole = rel_l2(G, ref["grads"])
    print(f"{name} F16 mask-free gradients: per tensor max {max(errs):.2e} (tensor {int(np.argmax(errs))}) "
          f"median {np.median(errs):.2e}; whole arena {whole:.2e}; all: {' '.join(f'{e:.1e}' for e in errs)}")
    for i, e in enumerate(errs):
        assert e < f16_grad_tol(i), f"tensor {i}: rel L2 {e:.3g} (bound {f16_grad_tol(i):.0e})"
    assert whole < 2e-3, f"whole gradient arena: rel L2 {whole:.3g}"
    model.close()


def test_config4_shard_vs_oracle(gpu, oracle):
    """Shard 5 of config 4's 65536-ray batch (8192 rays per GPU, global ids and global sum)."""
    import nof

    n, samples, shard = 8192, (128, 128), 5
    seed, step, base = 0x5EED0004, 1, shard * 8192
    r = _rays("blender", n, seed=45)
    msum = 8.0 * float(np.sum(r["lossmult"], dtype=np.float32))  # the 8 shards' global sum
    model = nof.AcceleratedMipNeRF(seed=13, max_rays=n, num_samples=samples)
    model.set_rng(seed, step, base)
    _gpu_step(model, r, gpu, msum)
    lv = [model.level_numpy(l) for l in range(2)]
    _check_t(oracle, lv, r, samples, seed, step, base)  # all 8192 rays
    # per-ray outputs of the shard's last 1024 rays (its tail blocks) vs the oracle's forward + adjoint
    lo = n - 1024
    sub = {k: v[lo:] for k, v in r.items()}
    ref = oracle.step(oracle.Spec(), nof.to_numpy(model.mlp.flat_params()[0], (546948,)), sub, samples=samples,
                      seed=seed, step_idx=step, ray_base=base + lo, loss_mult_sum=msum,
                      t_override={1: lv[1]["t"][lo:]}, nthreads=NTHREADS,
                      want=("sigma", "rgb", "w", "C", "dsigma", "drgb"))
    for l in range(2):
        for k in PER_RAY:
            e = rel_l2(lv[l][k][lo:], ref[ORACLE_KEY[k]][l])
            assert e < 1e-5, f"{k} level {l} (rays {lo}..{n - 1}): rel L2 {e:.3g}"
    # the gradient of a 1024-ray slice (same global ids and sum) vs the oracle, on the same model
    model.set_rng(seed, step, base + lo)
    _gpu_step(model, r, gpu, msum, lo, n)
    _compare_step(oracle, model, sub, samples, seed, step, base + lo, msum, 0)
    model.close()


@pytest.mark.parametrize("precision", [4, 0])
def test_persistent_groups_with_partial_tail(gpu, oracle, precision):
    """4 x CUs + 1 rays x 128+128 (1025 on a 256-CU part): 4 n sample blocks = 2 CUs + 1 groups of 8 per
    level, so the F16 kernels' persistent workgroup 0 (one per CU) runs three groups (0, CUs, 2 CUs) and the
    last is partial (4 blocks, its other waves duplicate the last block); the next groups' inputs are
    prefetched across group boundaries.
    Per-sample outputs do not depend on the grouping: the last 8 rays' forward outputs and integrator
    adjoint equal, bitwise, those of an 8-ray batch of the same rays (same global ids, same loss-mult sum,
    same parameters), and match the oracle's own forward within the mode's tolerance."""
    import nof

    import torch

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n, samples, tail = 4 * cus + 1, (128, 128), 8
    groups = -(-(n * samples[0] // 32) // 8)
    assert groups == 2 * cus + 1 and (n * samples[0] // 32) % 8 == 4, "three groups on workgroup 0, the last partial"
    seed, step, base = 0x5EED0007, 3, 4096
    r = _rays("blender", n, seed=77)
    msum = float(np.sum(r["lossmult"], dtype=np.float32))
    model = nof.AcceleratedMipNeRF(seed=5, max_rays=n, num_samples=samples, precision=precision)
    model.set_rng(seed, step, base)
    _gpu_step(model, r, gpu, msum)
    full = [model.level_numpy(l) for l in range(2)]
    _check_t(oracle, full, r, samples, seed, step, base)
    lo = n - tail
    params = nof.to_numpy(model.mlp.flat_params()[0], (546948,)).copy()
    small = nof.AcceleratedMipNeRF(seed=5, max_rays=tail, num_samples=samples, precision=precision)
    small.set_rng(seed, step, base + lo)
    _gpu_step(small, r, gpu, msum, lo, n)
    part = [small.level_numpy(l) for l in range(2)]
    for l in range(2):
        for k in PER_RAY + ("t",):
            assert np.array_equal(full[l][k][lo:], part[l][k]), f"{k} level {l}: grouping changed the result"
    sub = {k: v[lo:] for k, v in r.items()}
    ref = oracle.step(oracle.Spec(), params, sub, samples=samples, seed=seed, step_idx=step, ray_base=base + lo,
                      loss_mult_sum=msum, t_override={1: full[1]["t"][lo:]}, nthreads=NTHREADS,
                      want=tuple(ORACLE_KEY.values()))
    for l in range(2):
        for k in PER_RAY:
            e = rel_l2(full[l][k][lo:], ref[ORACLE_KEY[k]][l])
            assert e < TOLS[precision], f"{k} level {l} (rays {lo}..{n - 1}): rel L2 {e:.3g}"
    small.close()
    model.close()
