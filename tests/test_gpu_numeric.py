"""Runtime guards of the training step:

* non-finite detection: a NaN or inf reaching the integrator (sigma, rgb or the composite colour) sets
  NOF_NUMERIC_FORWARD (an fp16 activation overflow reaches it as an inf density); in the f16x2 perf mode a
  non-finite output gradient (which fmaxf would drop from the delta scale) sets NOF_NUMERIC_DELTA;
  clean steps report 0 and the bits clear on request;
* the per-kernel timer's event pool stays bounded when timing runs for many steps without a read,
  and the folded totals still count every launch.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _step(m, r, gpu):
    import torch

    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(gpu) for k, v in r.items()}
    n = r["o"].shape[0]
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
    torch.cuda.synchronize()


@pytest.mark.parametrize("precision", [0, 2, 3, 4])
def test_nonfinite_flags(gpu, precision):
    import nof
    from nof import synth

    n = 64
    m = nof.AcceleratedMipNeRF(seed=3, max_rays=n, num_samples=(64, 64), precision=precision)
    r = synth.blender_rays(n, seed=1)
    _step(m, r, gpu)
    assert m.numeric_status() == 0
    bad = {k: v.copy() for k, v in r.items()}
    # a NaN direction: its alphas and colour are NaN (a NaN origin would not do: the first ReLU,
    # v_max_f32(NaN, 0) = 0, drops it before the heads)
    bad["d"][5, 0] = np.nan
    _step(m, bad, gpu)
    st = m.numeric_status(clear=False)
    assert st & nof._lib.NOF_NUMERIC_FORWARD
    assert m.numeric_status(clear=True) == st  # read again, then cleared
    assert m.numeric_status() == 0
    if precision in (2, 3, 4):  # the f16 modes' delta scaling
        bad = {k: v.copy() for k, v in r.items()}
        bad["pix"][7, 1] = np.inf  # finite forward, non-finite output gradient
        _step(m, bad, gpu)
        st = m.numeric_status()
        assert st & nof._lib.NOF_NUMERIC_DELTA and not st & nof._lib.NOF_NUMERIC_FORWARD
    m.close()


def test_timer_pool_bounded(gpu):
    import torch
    import nof
    from nof import synth

    n = 32
    m = nof.AcceleratedMipNeRF(seed=1, max_rays=n, num_samples=(64, 64))
    r = synth.blender_rays(n, seed=2)
    d = {k: torch.from_numpy(v).to(gpu) for k, v in r.items()}
    m.enable_timing(True)
    steps = 400  # ~ 6400 timed launches: past the 4096-record bound, never read in between
    for _ in range(steps):
        m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
    t = m.read_timing()
    # one weight-gradient launch per step covers both levels
    assert t["mlp_fwd"][1] == 2 * steps and t["wgrad"][1] == steps and t["pack"][1] == steps
    assert all(ms > 0 for ms, cnt in t.values() if cnt)
    m.close()
