"""Multi-GPU data parallelism for vacv batches.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm, "gloo" for the CPU tests).  Images are independent, so a batch is
sharded by contiguous ranges with no data-path collective; the only exchange
is the global per-channel statistic: every rank reduces its
shard to (Sum x, Sum x^2) per channel (vacv_channel_sums, fp64, exact for u8
input), one all-reduce of 2*c doubles merges them, and every rank derives the
same mean / stddev.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """[begin, end) of this rank's contiguous share of `total` images
    (the first total % world ranks take one extra)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def allreduce_sums(local_sums: torch.Tensor, local_count: float, group=None) -> Tuple[torch.Tensor, float]:
    """Sum (c, 2) fp64 moment sums and the pixel count over all ranks."""
    buf = torch.cat([local_sums.reshape(-1).to(torch.float64),
                     torch.tensor([float(local_count)], dtype=torch.float64, device=local_sums.device)])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf[:-1].reshape(local_sums.shape), float(buf[-1].item())


def allreduce_sums_async(local_sums: torch.Tensor, local_count: float, group=None):
    """allreduce_sums without a host round trip: the count stays a device
    tensor, so a step that all-reduces its statistics never synchronises."""
    buf = torch.cat([local_sums.reshape(-1).to(torch.float64),
                     torch.full((1,), float(local_count), dtype=torch.float64, device=local_sums.device)])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf[:-1].reshape(local_sums.shape), buf[-1]


def stats_from_moments(sums: torch.Tensor, count: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Host-side twin of vacv_stats_from_sums (same formula) for any device."""
    s = sums.reshape(-1, 2).to(torch.float64)
    mean = s[:, 0] / count
    var = torch.clamp(s[:, 1] / count - mean * mean, min=0.0)
    return mean.to(torch.float32), torch.sqrt(var).to(torch.float32)


def global_mean_stddev(shard: torch.Tensor, layout: int = 1, group=None):
    """Global per-channel mean/stddev of a batch sharded over the ranks.

    `shard` is this rank's (n_local, ...) device batch.  Returns float32 (c,)
    tensors, identical on every rank."""
    from . import ops
    from ._lib import NHWC
    sums = ops.channel_sums(shard, per_image=False, layout=layout)[0]  # (c, 2)
    s4 = ops._as4d(shard, layout)
    h, w = (s4.shape[1], s4.shape[2]) if layout == NHWC else (s4.shape[2], s4.shape[3])
    total, count = allreduce_sums(sums, float(s4.shape[0]) * h * w, group)
    return stats_from_moments(total, count)
