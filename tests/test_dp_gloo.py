"""World-size-2 data-parallel logic on CPU (gloo): sharded gradients with global ray ids and the
global loss-multiplier sum, all-reduced bucket by bucket in the overlapped path's order, equal the
single-process gradient of the whole batch.
The per-shard compute is the oracle (there is no GPU here); the sharding, normalisation and
collective are the product's (nof.dp + torch.distributed), exactly as bench.py uses them."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SPEC = dict(D=4, W=32, Dc=1, Wc=16)
SAMPLES = (64, 64)


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle"), os.path.join(root, "nerf-or-nothing_amd")]
    import torch
    import torch.distributed as dist

    import oracle as O
    from nof import dp, synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = O.Spec(**SPEC)
    P = O.glorot_init(spec, 9)
    rays = synth.blender_rays(7, seed=4)  # odd size: uneven shards
    rays["lossmult"] = np.linspace(0.5, 1.5, 7).astype(np.float32)
    shard, base = dp.shard_batch(rays, world, rank)
    out = O.step(spec, P, shard, samples=SAMPLES, seed=11, step_idx=2, ray_base=base,
                 loss_mult_sum=dp.global_loss_mult_sum(rays), nthreads=1, want=("grads",))
    g = torch.from_numpy(out["grads"])
    # the bucketed order of the overlapped all-reduce (nof.dp.BucketedAllReduce): bucket 0 (the
    # layers whose weight gradients finish first) then bucket 1, each over its arena spans
    sizes = [int(x) for x in O.layer_sizes(spec)]
    import nof

    for b in range(2):
        for off, cnt in nof.grad_bucket_spans(sizes, b):
            dist.all_reduce(g[off:off + cnt])
    loss = torch.tensor([out["loss"]], dtype=torch.float64)
    dist.all_reduce(loss)
    if rank == 0:
        q.put((g.numpy(), float(loss.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_allreduce_equals_full_batch(oracle):
    import torch.multiprocessing as mp

    from nof import dp, synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g, loss = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = oracle.Spec(**SPEC)
    P = oracle.glorot_init(spec, 9)
    rays = synth.blender_rays(7, seed=4)
    rays["lossmult"] = np.linspace(0.5, 1.5, 7).astype(np.float32)
    ref = oracle.step(spec, P, rays, samples=SAMPLES, seed=11, step_idx=2, ray_base=0, nthreads=1, want=("grads",))
    assert np.linalg.norm(g - ref["grads"]) <= 1e-12 * np.linalg.norm(ref["grads"])
    assert abs(loss - ref["loss"]) <= 1e-12 * abs(ref["loss"])


@pytest.mark.parametrize("n,world", [(1024, 8), (7, 2), (5, 4), (1, 1)])
def test_shard_ranges_partition(n, world):
    from nof import dp

    rs = [dp.shard_range(n, world, r) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
    sizes = [e - b for b, e in rs]
    assert max(sizes) - min(sizes) <= 1


def _sync_worker(rank, world, port, perturb, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "nerf-or-nothing_amd")]
    import torch
    import torch.distributed as dist

    from nof import dp

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = torch.from_numpy(np.random.default_rng(3).standard_normal(546948).astype(np.float32))
    if perturb and rank == 1:  # one ulp of one parameter on one rank
        p[1234] = torch.from_numpy(np.nextafter(p[1234:1235].numpy(), np.float32(np.inf)))
    q.put((rank, dp.params_in_sync(p)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("perturb", [False, True])
def test_params_in_sync_across_ranks(perturb):
    """SURVEY §8e's periodic parameter assertion (nof.dp.params_in_sync, the Trainer's
    sync_check_every): every rank agrees the replicas are identical, and a one-ulp difference on one
    rank is reported on every rank."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sync_worker, args=(r, 2, port, perturb, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: not perturb, 1: not perturb}
