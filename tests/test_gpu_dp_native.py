"""The C ABI's native RCCL data parallelism (nof_dp_*) on the one GPU of the box: world size 1
(a multi-rank communicator needs distinct GPUs).  All-reduce of one rank is the identity, so the
gradient arena must come back bit-identical; the grouped single-process path likewise."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _step(gpu, seed):
    import torch
    import nof
    from nof import synth

    n = 64
    r = synth.blender_rays(n, seed=seed)
    d = {k: torch.from_numpy(v).to(gpu) for k, v in r.items()}
    m = nof.AcceleratedMipNeRF(seed=3, max_rays=n, num_samples=(64, 64))
    m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"], float(n))
    torch.cuda.synchronize()
    return m


def test_native_dp_world1_identity(gpu):
    import torch
    import nof
    from nof.dp import NativeDP

    m = _step(gpu, 1)
    g0 = nof.to_numpy(m.mlp.flat_grads()[0], (546948,)).copy()
    dp = NativeDP.init_rank(NativeDP.unique_id(), 1, 0, 0)
    dp.allreduce_grads(m)
    torch.cuda.synchronize()
    assert np.array_equal(nof.to_numpy(m.mlp.flat_grads()[0], (546948,)), g0)
    t = torch.arange(1000, dtype=torch.float32, device=gpu)
    dp.allreduce(t.data_ptr(), 1000)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(1000, dtype=torch.float32, device=gpu))
    dp.close()
    (d1,) = NativeDP.init_all([0])
    NativeDP.allreduce_grads_all([d1], [m])
    torch.cuda.synchronize()
    assert np.array_equal(nof.to_numpy(m.mlp.flat_grads()[0], (546948,)), g0)
    d1.close()
    m.close()


def test_step_end_waits_one_step_behind(gpu):
    """nof_dp_step_end: each call waits, boundedly, for the PREVIOUS step's all-reduces;
    a final nof_dp_wait covers the last.  Loopback group of two on the one GPU: 1, 2 -> 3 -> 6 -> 12."""
    import torch
    import nof
    from nof.dp import NativeDP

    dps = NativeDP.init_loopback(2, 0)
    ts = [torch.full((1000,), float(i + 1), device=gpu) for i in range(2)]
    for _ in range(3):
        for d, t in zip(dps, ts):
            d.allreduce(t.data_ptr(), 1000)
        for d in dps:
            d.step_end()
    for d in dps:
        d.wait()
    torch.cuda.synchronize()
    for t in ts:
        assert torch.equal(t, torch.full((1000,), 12.0, device=gpu))
    dps[0].abort()
    with pytest.raises(nof.NofError):
        dps[0].step_end()
    for d in dps:
        d.close()


def test_wait_after_step_end_covers_the_last_step(gpu):
    """after nof_dp_step_end the step's all-reduce is the LAGGED one; a final nof_dp_wait must
    still wait for it (boundedly).  The all-reduce sits behind a ~0.5 s spin on the stream, so a wait with a
    50 ms limit has to time out and fail loudly instead of returning at once."""
    import torch
    import nof
    from nof.dp import NativeDP

    dps = NativeDP.init_loopback(2, 0)
    ts = [torch.full((1000,), float(i + 1), device=gpu) for i in range(2)]
    torch.cuda._sleep(1_000_000_000)  # ~0.5 s of GPU clock ticks ahead of the all-reduce on the null stream
    for d, t in zip(dps, ts):
        d.allreduce(t.data_ptr(), 1000)
    for d in dps:
        d.step_end()  # no earlier step: returns at once; this step becomes the lagged one
    with pytest.raises(nof.NofError):
        dps[0].wait(50)
    torch.cuda.synchronize()
    dps[1].wait(60000)  # the other member's lagged all-reduce has completed by now
    for t in ts:
        assert torch.equal(t, torch.full((1000,), 3.0, device=gpu))
    for d in dps:
        d.close()
