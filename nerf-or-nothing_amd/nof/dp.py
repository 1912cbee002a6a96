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
