"""The native data-parallel choreography with K > 1 models on ONE GPU (SURVEY.md §4 "T0 DP logic",
VERDICT r2 items 4-5): a loopback group (nof_dp_init_loopback) stands in for RCCL — its all-reduce is a
device sum of the members' arenas in member order — so the grouped all-reduce, the gradient-bucket hook
(nof_dp_attach: reverse-layer spans, the last member's arrival releasing every replica's stream),
micro-batch accumulation and the one-call nof_dp_train_step all run for real before any multi-GPU node:

  * K shards with global ray ids + the global loss-multiplier sum + the all-reduce == the single-model
    gradient of the whole batch (fp32 accuracy: the shard sums are added in another order);
  * after Adam every replica holds bitwise-identical parameters;
  * nof_dp_train_step at N = 1 == the Python Trainer bit for bit, and at K = 2 == the same step
    emulated in Python (two shard gradients added by torch, Adam) bit for bit;
  * bin/nof_train --gpus 2 --dp loopback [--micro-batch] == --gpus 1 to fp32 accuracy, and --attach ==
    the grouped all-reduce bit for bit (bucket-aligned weight-gradient items, nof_config.grad_buckets).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "nerf-or-nothing_amd", "bin", "nof_train")
SAMPLES = (64, 64)
SEED = 0x77


def _records(n, seed):
    from nof import synth

    r = synth.blender_rays(n, seed=seed)
    r["lossmult"] = np.random.default_rng(seed).uniform(0.5, 1.5, n).astype(np.float32)
    return synth.pack_records(r)


# the any-shape path's network (configs[0]: 4x128): its 2L-tensor arena through the same all-reduce
NETS = {"ref": {}, "4x128": dict(net_depth=4, net_width=128)}


def _models(k, max_rays, precision=0, grad_buckets=0, net="ref"):
    import nof

    ms = [nof.AcceleratedMipNeRF(seed=SEED, max_rays=max_rays, num_samples=SAMPLES, precision=precision,
                                 grad_buckets=grad_buckets, **NETS[net]) for _ in range(k)]
    return ms, [nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config) for m in ms]


def _flat(m, which):
    import nof

    ptr, P = m.mlp.flat_grads() if which == "g" else m.mlp.flat_params()
    return nof.to_numpy(ptr, (P,)).copy()


def _grad(m, ds, n, step, ray_base, msum, accumulate=False, publish=True):
    b, _ = ds.next(n, SEED, step, ray_base)
    p = {k: v[0] for k, v in b.items()}
    m.set_rng(SEED, step, ray_base)
    m.get_gradient_device(n, p["o"], p["d"], p["radius"], p["near"], p["far"], p["lossmult"], p["pix"], msum,
                          accumulate=accumulate, publish=publish)


@pytest.mark.parametrize("net", list(NETS))
@pytest.mark.parametrize("mode", ["grouped", "attached"])
def test_loopback_k2_equals_single_model(gpu, mode, net):
    import torch
    import nof
    from nof.dp import NativeDP

    B, K, step = 256, 2, 3
    ds = nof.RayDataset(records=_records(3000, 5))
    _, msum = ds.next(B, SEED, step, 0)
    single, sadam = _models(1, B, net=net)
    _grad(single[0], ds, B, step, 0, msum)
    torch.cuda.synchronize()
    g_full = _flat(single[0], "g")

    sh = B // K
    ms, adams = _models(K, sh, net=net)
    dps = NativeDP.init_loopback(K, 0)
    try:
        if mode == "attached":
            for d, m in zip(dps, ms):
                d.attach(m)
        for r, m in enumerate(ms):  # global ray ids, the GLOBAL loss-multiplier sum
            _grad(m, ds, sh, step, r * sh, msum)
        if mode == "grouped":
            NativeDP.allreduce_grads_all(dps, ms)
        for d in dps:
            d.wait()
        torch.cuda.synchronize()
        gs = [_flat(m, "g") for m in ms]
        assert np.array_equal(gs[0], gs[1]), "the replicas' all-reduced gradients differ"
        assert rel_l2(gs[0], g_full) <= 1e-5
        lr = nof.learning_rate_decay(step)
        for m, o in zip(ms, adams):
            o.step(m.mlp.allParams, m.mlp.allGradients, lr)
        torch.cuda.synchronize()
        assert np.array_equal(_flat(ms[0], "p"), _flat(ms[1], "p"))
    finally:
        for d in dps:
            if mode == "attached":
                d.attach(None)
            d.close()
        for m in ms + single:
            m.close()


def test_loopback_missing_member_fails_loudly(gpu):
    import nof
    from nof.dp import NativeDP

    ms, _ = _models(2, 64)
    dps = NativeDP.init_loopback(2, 0)
    ptr, P = ms[0].mlp.flat_grads()
    dps[0].allreduce(ptr, P)  # member 1 never arrives
    with pytest.raises(nof.NofError):
        dps[0].wait(1000)
    with pytest.raises(nof.NofError):  # the aborted member stays aborted
        dps[0].allreduce(ptr, P)
    for d in dps:
        d.close()
    for m in ms:
        m.close()


def test_attached_model_destroyed_before_detach(gpu):
    """destroying a model while attached must not leave the communicator pointing at it."""
    import torch
    from nof.dp import NativeDP

    ms, _ = _models(1, 64)
    dps = NativeDP.init_loopback(1, 0)
    dps[0].attach(ms[0])
    ms[0].close()  # destroys the native model while attached
    dps[0].abort()  # would touch the freed model before the fix
    dps[0].close()
    torch.cuda.synchronize()


def test_train_step_n1_matches_python_trainer(gpu, tmp_path):
    import torch
    import nof
    from nof import dp as ndp
    from nof.train import Trainer

    path = tmp_path / "train.bin"
    _records(4000, 13).tofile(path)
    tr = Trainer(nof.RayDataset(path), batch_size=256, seed=77, print_every=0)
    tr.train(3)
    m = nof.AcceleratedMipNeRF(tr.cfg)  # the Trainer's config (default sample counts)
    a = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)
    ds = nof.RayDataset(path)
    for step in range(1, 4):
        ndp.train_step(None, [m], [a], [ds], 256, step, nof.learning_rate_decay(step, **tr.lr), seed=77)
    torch.cuda.synchronize()
    assert np.array_equal(_flat(m, "p"), _flat(tr.model, "p"))


@pytest.mark.parametrize("micro,attach", [(0, False), (64, False), (64, True)])
def test_train_step_loopback_k2_matches_emulation(gpu, micro, attach):
    """K = 2 through nof_dp_train_step == the same step written out in Python: each replica's shard in
    micro-batches (accumulated), the two arenas added by torch (g0 + g1, the loopback order), Adam."""
    import torch
    import nof
    from nof import dp as ndp
    from nof.dp import NativeDP

    B, K = 256, 2
    sh = B // K
    mb = micro or sh
    ds_py = nof.RayDataset(records=_records(3000, 9))
    # bucket-aligned weight-gradient items (nof_config.grad_buckets; an attached model selects them): the
    # unbucketed emulation then sums every gradient element exactly as the bucketed launches do
    ms_py, ad_py = _models(K, mb, grad_buckets=1)
    ms, ad = _models(K, mb, grad_buckets=1)
    dss = [nof.RayDataset(records=_records(3000, 9)) for _ in range(K)]
    dps = NativeDP.init_loopback(K, 0)
    if attach:
        for d, m in zip(dps, ms):
            d.attach(m)
    try:
        for step in (1, 2):
            lr = nof.learning_rate_decay(step)
            msum_native = ndp.train_step(dps, ms, ad, dss, B, step, lr, seed=SEED, micro_batch=micro)
            msum = np.float32(0.0)
            for r in range(K):
                for j in range(sh // mb):
                    _, s = ds_py.next(mb, SEED, step, r * sh + j * mb)
                    msum = np.float32(msum + np.float32(s))
            assert msum_native == float(msum)
            for r, m in enumerate(ms_py):
                for j in range(sh // mb):
                    _grad(m, ds_py, mb, step, r * sh + j * mb, float(msum), accumulate=j > 0)
            torch.cuda.synchronize()
            g = [nof.device_tensor(m.mlp.flat_grads()[0], (m.mlp.flat_grads()[1],), device=torch.device("cuda", 0))
                 for m in ms_py]
            tot = g[0] + g[1]
            for t in g:
                t.copy_(tot)
            torch.cuda.synchronize()
            for m, o in zip(ms_py, ad_py):
                o.step(m.mlp.allParams, m.mlp.allGradients, lr)
            torch.cuda.synchronize()
            for r in range(K):
                assert np.array_equal(_flat(ms[r], "p"), _flat(ms_py[r], "p")), f"replica {r} step {step}"
            assert np.array_equal(_flat(ms[0], "p"), _flat(ms[1], "p"))
    finally:
        for d in dps:
            if attach:
                d.attach(None)
            d.close()
        for m in ms + ms_py:
            m.close()


@pytest.mark.parametrize("micro", [[], ["--micro-batch", 64]])
def test_native_driver_loopback_equals_one_replica(gpu, tmp_path, micro):
    """--gpus 2 --dp loopback == --gpus 1 to fp32 accuracy (the shards' sums add in another order), and
    --attach (bucketed all-reduce through the hook) == the grouped all-reduce BIT FOR BIT: a data-parallel
    driver cuts the weight-gradient items per bucket (nof_config.grad_buckets)."""
    path = tmp_path / "train.bin"
    _records(4000, 13).tofile(path)
    common = [EXE, "--records", path, "--batch", 256, "--seed", 77, "--print-every", 0, "--steps", 3]
    run = lambda *a: subprocess.run([str(x) for x in (*common, *a)], capture_output=True, text=True, timeout=120)
    one = run("--gpus", 1, "--dump-params", tmp_path / "p1.bin")
    assert one.returncode == 0, one.stderr[-2000:]
    p1 = np.fromfile(tmp_path / "p1.bin", np.float32)
    p2 = {}
    for mode in ("grouped", "attach"):
        extra = list(micro) + (["--attach"] if mode == "attach" else [])
        two = run("--gpus", 2, "--dp", "loopback", *extra, "--dump-params", tmp_path / f"p2{mode}.bin")
        assert two.returncode == 0, two.stderr[-2000:]
        assert "parameters identical on 2 devices" in two.stdout  # the driver's own replica check
        p2[mode] = np.fromfile(tmp_path / f"p2{mode}.bin", np.float32)
        assert rel_l2(p2[mode], p1) <= 1e-6
    assert np.array_equal(p2["attach"], p2["grouped"]), "attached and grouped data parallelism differ"
