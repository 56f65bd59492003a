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

import contextlib
from typing import Dict, List, Optional, Tuple

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


class OverlappedGradAllReduce:
    """The gradient average, overlapped with the backward: each encoder layer's gradient region
    (one contiguous ~5 MB slice of the flat buffer at C4) is all-reduced as soon as its backward
    has been enqueued, on RCCL's stream ordered after the stream that writes those gradients
    (the executor's side stream), while the next layer's backward runs; the remaining regions
    (the head) go at the end of the step, then the step's main stream waits for every
    collective and scales by 1/world.  Same result as GradAllReduce (sum of the same per-rank
    buffers by the same collective, then one scaling), each rank issuing the same sequence.

    Wiring: ``stack.grad_ready = ar.layer_done`` (EncoderStack calls it with the layer's
    parameter-name prefix and the stream that wrote its gradients) and ``trainer.grad_sync = ar``.
    """

    def __init__(self, flat, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.flat = flat
        base = flat.gflat.data_ptr()
        self.span: Dict[str, Tuple[int, int]] = {}
        for name in flat.names:
            g = flat.grads[name]
            lo = (g.data_ptr() - base) // 4
            self.span[name] = (lo, lo + g.numel())
        self.pending: List = []
        self.launched: List[Tuple[int, int]] = []

    def region(self, prefix: str) -> Tuple[int, int]:
        """Element range [lo, hi) of the parameters named prefix*, which must be contiguous."""
        r = sorted(v for k, v in self.span.items() if k.startswith(prefix))
        if not r:
            raise KeyError(prefix)
        lo, hi = r[0][0], r[-1][1]
        covered = sum(b - a for a, b in r)
        inside = sum(b - a for k, (a, b) in self.span.items() if a >= lo and b <= hi)
        if covered != inside:
            raise ValueError(f"parameters {prefix}* are not contiguous in the flat buffer")
        return lo, self._align_end(hi)

    def _align_end(self, hi: int) -> int:
        # the flat buffer pads every parameter to 4 floats: include the padding up to the next one
        nxt = [a for a, _ in self.span.values() if a >= hi]
        return min(nxt) if nxt else self.flat.gflat.numel()

    def layer_done(self, prefix: str, stream: Optional["torch.cuda.Stream"] = None) -> None:
        lo, hi = self.region(prefix)
        g = self.flat.gflat
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            self.pending.append(self.dist.all_reduce(g[lo:hi], group=self.group, async_op=True))
        self.launched.append((lo, hi))

    def __call__(self, flat) -> None:
        g = flat.gflat
        o = 0
        for lo, hi in sorted(self.launched) + [(g.numel(), g.numel())]:
            if lo > o:   # a region no layer_done covered (head parameters, padding)
                self.pending.append(self.dist.all_reduce(g[o:lo], group=self.group, async_op=True))
            o = max(o, hi)
        for h in self.pending:
            h.wait()
        self.pending.clear()
        self.launched.clear()
        g.mul_(1.0 / self.world)


def broadcast_params(flat, src: int = 0, group=None) -> None:
    import torch.distributed as dist
    dist.broadcast(flat.flat, src, group=group)
