"""Edge cases of the training step on the GPU, through the C ABI, against the fp64 oracle:
a single ray, the largest per-level sample count (512), a ray count that leaves a partly filled
workgroup, a fine level with fewer samples than the coarse one, masked rays (lossmult = 0), and the
argument errors the boundary reports instead of launching (n = 0, n > max_rays, a zero loss-mult
sum, an unsupported sample count)."""
import ctypes as C

import numpy as np
import pytest

import test_gpu_step as step_tests
from conftest import rel_l2

pytestmark = pytest.mark.gpu


# (n, samples): one ray (two 32-sample blocks of a 4-block workgroup), one ray at 512 + 512
# samples (8 values per lane in the integrator, 16 blocks), 5 rays x 128 + 64 (the fine level
# smaller than the coarse one: resampling 128 -> 64)
@pytest.mark.parametrize("precision", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n,samples", [(1, (64, 64)), (1, (512, 512)), (5, (128, 64))])
def test_step_parity_edges(gpu, oracle, n, samples, precision):
    step_tests.test_step_parity(gpu, oracle, "blender", n, samples, precision)


@pytest.mark.parametrize("precision", [0, 2, 3, 4])
def test_masked_rays(gpu, oracle, precision):
    """lossmult = 0 rays (BinDataset records may carry any lossmult, MNcs:136-140): they add nothing to
    the loss or the gradient, and the loss normalises by the sum over the rest (D14)."""
    import torch
    import nof
    from nof import synth

    n, samples, seed, step = 12, (64, 128), 0x77, 2
    r = synth.blender_rays(n, seed=21)
    r["lossmult"] = np.array([1.0, 0.0, 2.0, 0.0] * 3, np.float32)
    model = nof.AcceleratedMipNeRF(seed=seed, max_rays=n, num_samples=samples, precision=precision)
    model.set_rng(seed, step, 0)
    step_tests._run_gpu(model, r, gpu)
    torch.cuda.synchronize()
    lv = [model.level_numpy(l) for l in range(2)]
    for l in range(2):  # masked rays: exactly zero output gradients
        assert not np.any(lv[l]["density_grad"][r["lossmult"] == 0])
        assert not np.any(lv[l]["rgb_grad"][r["lossmult"] == 0])
        assert np.any(lv[l]["density_grad"][r["lossmult"] > 0])
    pptr, P = model.mlp.flat_params()
    params = nof.to_numpy(pptr, (P,))
    G = nof.to_numpy(model.mlp.flat_grads()[0], (P,))
    masks = {l: model.mlp.relu_masks(l).reshape(n, samples[l], -1) for l in range(2)}
    ref = oracle.step(oracle.Spec(), params, r, samples=samples, seed=seed, step_idx=step, ray_base=0,
                      t_override={1: lv[1]["t"]}, relu_mask=masks, nthreads=16)
    tol = step_tests.TOLS[precision]
    assert rel_l2(G, ref["grads"]) < tol
    assert abs(model.loss() - ref["loss"]) <= tol * abs(ref["loss"])
    model.close()


def test_boundary_argument_errors(gpu):
    """The C ABI rejects bad calls with NOF_ERR_INVALID_ARG (1) before any launch, and a bad config
    with NOF_ERR_UNSUPPORTED (5); the object stays usable afterwards."""
    import torch
    import nof
    from nof import synth

    n = 4
    r = synth.blender_rays(n, seed=3)
    d = step_tests._device_rays(r, gpu)
    model = nof.AcceleratedMipNeRF(seed=1, max_rays=n, num_samples=(64, 64))
    args = (d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"])
    for bad_n, msum in ((0, 4.0), (n + 1, 4.0), (-1, 4.0), (n, 0.0)):
        with pytest.raises(nof.NofError) as e:
            model.get_gradient_device(bad_n, *args, msum)
        assert e.value.status == 1, (bad_n, msum)
    with pytest.raises(nof.NofError) as e:
        model.render_device(0, *args[:5])
    assert e.value.status == 1
    cfg = nof.default_config(num_samples=(64, 192))
    h = C.c_void_p()
    assert nof.lib().nof_mipnerf_create(C.byref(cfg), C.byref(h)) == 5
    model.get_gradient_device(n, *args, 4.0)  # still usable
    torch.cuda.synchronize()
    assert np.isfinite(model.loss())
    model.close()
