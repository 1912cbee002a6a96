"""Data-parallel sharding of ray batches.

Rays are independent; the only cross-ray coupling of the step is the loss normalisation
sum m_r (AF:356: dL/dC = 2 m / sum m (C - p)) and the gradient sum over rays.  So each rank
takes a contiguous shard of the global batch, keeps GLOBAL ray ids (the Philox counter uses
them, so a sample never depends on the sharding), normalises by the GLOBAL sum of loss
multipliers, and the per-rank gradient sums are added with one all-reduce (no averaging:
the loss is a sum over rays).  Parameters stay bitwise identical across ranks because every
rank applies Adam to the same all-reduced bits.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_global: int, world: int, rank: int) -> tuple[int, int]:
    """[begin, end) of rank's contiguous shard; sizes differ by at most one ray."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    base, extra = divmod(n_global, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def shard_batch(rays: dict, world: int, rank: int) -> tuple[dict, int]:
    """(rank's shard of a global SoA batch, global id of its first ray)."""
    n = next(iter(rays.values())).shape[0]
    b, e = shard_range(n, world, rank)
    return {k: np.ascontiguousarray(v[b:e]) for k, v in rays.items()}, b


def global_loss_mult_sum(rays: dict) -> float:
    """sum of loss multipliers over the WHOLE batch, accumulated in float as the reference
    intends (it truncates to int, MNcpp:61-65, D14)."""
    return float(np.sum(np.asarray(rays["lossmult"], np.float32), dtype=np.float32))


def params_checksum(flat):
    """Order-sensitive checksum of a flat fp32 parameter tensor (any device): sum over i of
    (i + 1) * bits(p_i) in wrapping int64 — equal on two ranks iff (with overwhelming probability)
    their parameters are bitwise equal.  Returns a 1-element int64 tensor on flat's device."""
    import torch

    bits = flat.contiguous().view(torch.int32).to(torch.int64)
    idx = torch.arange(1, bits.numel() + 1, device=bits.device, dtype=torch.int64)
    return (bits * idx).sum().reshape(1)


def params_in_sync(flat, allreduce=None) -> bool:
    """SURVEY §8e's data-parallel invariant, checked across ranks: every rank applies Adam to the
    same all-reduced gradient bits, so the parameters must stay bitwise identical.  One all-reduce
    (MAX) of (checksum, -checksum): equal on every rank iff max == min.  `allreduce(t, op)`
    defaults to torch.distributed.all_reduce (the trainers pass their own for gloo rehearsals)."""
    import torch
    import torch.distributed as dist

    cs = params_checksum(flat)
    both = torch.cat([cs, -cs])
    if allreduce is None:
        dist.all_reduce(both, op=dist.ReduceOp.MAX)
    else:
        allreduce(both, dist.ReduceOp.MAX)
    return bool(both[0].item() == -both[1].item())


class NativeDP:
    """The C ABI's RCCL data parallelism (nof_dp_*, include/nof.h) for hosts without
    torch.distributed: one in-place all-reduce (sum) of the gradient arena per step."""

    def __init__(self, handle):
        self._h = handle
        self._model = None  # the attached model, kept alive while attached

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        from ._lib import call

        buf = (C.c_uint8 * 128)()
        call("nof_dp_unique_id", buf)
        return bytes(buf)

    @classmethod
    def init_rank(cls, uid: bytes, world: int, rank: int, device: int, timeout_ms: int = 0) -> "NativeDP":
        """Non-blocking communicator: waits at most timeout_ms (0 = NOF_DP_TIMEOUT_MS or 300 s) for
        every rank, then aborts (NofError NOF_ERR_RCCL)."""
        import ctypes as C
        from ._lib import call

        h = C.c_void_p()
        call("nof_dp_init_rank_timeout", (C.c_uint8 * 128).from_buffer_copy(uid), world, rank, device, timeout_ms,
             C.byref(h))
        return cls(h)

    @classmethod
    def init_loopback(cls, k: int, device: int = 0) -> list:
        """k communicators on ONE device whose all-reduce is a device sum in member order (SURVEY §4's
        loopback backend): the native DP choreography with k models on one GPU."""
        import ctypes as C
        from ._lib import call

        hs = (C.c_void_p * k)()
        call("nof_dp_init_loopback", k, device, hs)
        return [cls(C.c_void_p(h)) for h in hs]

    @classmethod
    def init_all(cls, devices) -> list:
        import ctypes as C
        from ._lib import call

        n = len(devices)
        hs = (C.c_void_p * n)()
        call("nof_dp_init_all", n, (C.c_int32 * n)(*devices), hs)
        return [cls(C.c_void_p(h)) for h in hs]

    def allreduce(self, ptr: int, count: int, stream=None):
        from ._lib import call

        call("nof_dp_allreduce", self._h, ptr, count, stream)

    def allreduce_grads(self, model, stream=None):
        from ._lib import call

        call("nof_dp_allreduce_grads", self._h, model._h, stream)

    @staticmethod
    def allreduce_grads_all(dps, models, streams=None):
        import ctypes as C
        from ._lib import call

        n = len(dps)
        st = (C.c_void_p * n)(*(streams or [None] * n))
        call("nof_dp_allreduce_grads_all", n, (C.c_void_p * n)(*[d._h.value for d in dps]),
             (C.c_void_p * n)(*[m._h.value for m in models]), st)

    def attach(self, model, comm_stream=None):
        """Overlapped mode: each publishing get_gradient call all-reduces the gradient buckets on
        comm_stream as they complete; the model's stream waits for the last (model=None detaches)."""
        from ._lib import call

        call("nof_dp_attach", self._h, model._h if model is not None else None, comm_stream)
        self._model = model

    def wait(self, timeout_ms: int = 0):
        """Failure detection: block until the last all-reduce is done; an RCCL error or a timeout
        aborts the communicator and raises NofError (NOF_ERR_RCCL)."""
        from ._lib import call

        call("nof_dp_wait", self._h, timeout_ms)

    def step_end(self, timeout_ms: int = 0):
        """nof_dp_step_end: the bounded wait of wait(), one step behind (the previous step's
        all-reduces), so the host enqueues the next step meanwhile; a final wait() covers the last."""
        from ._lib import call

        call("nof_dp_step_end", self._h, timeout_ms)

    def abort(self):
        from ._lib import call

        call("nof_dp_abort", self._h)

    def close(self):
        if getattr(self, "_h", None):
            from ._lib import lib

            lib().nof_dp_destroy(self._h)
            self._h = None
            self._model = None


def train_step(dps, models, adams, datasets, global_batch: int, step: int, lr: float, seed: int,
               micro_batch: int = 0) -> float:
    """nof_dp_train_step (include/nof.h): one data-parallel TrainStep over len(models) replicas —
    shards with global ray ids, the global loss-multiplier sum, micro-batch accumulation, the gradient
    all-reduce, Adam and a bounded wait; dps = None: one replica, no exchange.  Returns the global sum."""
    import ctypes as C
    from ._lib import call

    n = len(models)
    msum = C.c_float()
    dph = (C.c_void_p * n)(*[d._h.value for d in dps]) if dps else None
    call("nof_dp_train_step", n, dph, (C.c_void_p * n)(*[m._h.value for m in models]),
         (C.c_void_p * n)(*[a._h.value for a in adams]), (C.c_void_p * n)(*[d._h.value for d in datasets]),
         global_batch, micro_batch, seed, step, lr, C.byref(msum))
    return msum.value


class BucketedAllReduce:
    """torch.distributed (RCCL) all-reduce of the gradient arena, bucket by bucket, overlapped with
    the rest of the backward: installed as the model's gradient-bucket hook (include/nof.h
    nof_mipnerf_set_grad_buckets).  Each bucket's all-reduce is enqueued on a communication stream
    behind the model's stream; after the last bucket the model's stream waits for the
    communication stream, so Adam (or anything else enqueued on it) sees the reduced gradient.
    `allreduce(tensor)` defaults to dist.all_reduce (sum)."""

    def __init__(self, model, device, allreduce=None):
        import torch
        import torch.distributed as dist

        from .api import device_tensor

        self.model = model
        self.device = torch.device(device)
        st = model.config.stream
        self.lib_stream = (torch.cuda.ExternalStream(st, device=self.device) if st
                           else torch.cuda.default_stream(self.device))
        self.comm = torch.cuda.Stream(self.device)
        gptr, P = model.mlp.flat_grads()
        self.grad = device_tensor(gptr, (P,), device=self.device)
        self.allreduce = allreduce or dist.all_reduce
        self.buckets_seen = []
        model.set_grad_buckets(self._hook)

    def _hook(self, bucket, spans):
        import torch

        from ._lib import NOF_GRAD_BUCKETS

        self.buckets_seen.append(bucket)
        self.comm.wait_stream(self.lib_stream)
        with torch.cuda.stream(self.comm):
            for off, cnt in spans:
                self.allreduce(self.grad[off:off + cnt])
        if bucket == NOF_GRAD_BUCKETS - 1:
            self.lib_stream.wait_stream(self.comm)

    def close(self):
        self.model.set_grad_buckets(None)
