"""Data parallelism over the GPUs of one node: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm, over xGMI); gloo works for CPU tests of the same code.

Partitioning: a global step is G consecutive batches of the reference's single
numpy stream; rank r assembles batch r and *replays* (consumes without building) the others, so
the union of the ranks' batches is exactly what a single process would train on G steps.  A
64-graph batch never splits across GPUs (attention couples all graphs of a batch).

The only collective is the gradient all-reduce (average) over the flat fp32 gradient buffer,
issued in a few large buckets: xGMI is point-to-point (7 links per GPU), so RCCL's ring/tree
bandwidth per collective is what matters, and a handful of multi-MB buckets keeps it link-bound
rather than latency-bound.  Clip + Adam then run redundantly (bit-identically) on every rank.
"""
from __future__ import annotations

from typing import List

import torch


def rank_batches(loader, world: int, rank: int, n_steps: int) -> List:
    """The HostBatches rank `rank` trains on for `n_steps` global steps."""
    out = []
    for _ in range(n_steps):
        for g in range(world):
            if g == rank:
                out.append(loader())
            else:
                loader.replay()
    return out


class GradAllReduce:
    """Average the flat gradient buffer over the process group in `bucket_mb` chunks."""

    def __init__(self, group=None, bucket_mb: float = 8.0):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket = max(1, int(bucket_mb * (1 << 20) // 4))

    def __call__(self, flat) -> None:
        g = flat.gflat
        handles = []
        for o in range(0, g.numel(), self.bucket):
            handles.append(self.dist.all_reduce(g[o:o + self.bucket], group=self.group, async_op=True))
        for h in handles:
            h.wait()
        g.mul_(1.0 / self.world)


def broadcast_params(flat, src: int = 0, group=None) -> None:
    import torch.distributed as dist
    dist.broadcast(flat.flat, src, group=group)
