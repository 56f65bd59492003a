"""Data parallelism over the GPUs of one node: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm, over xGMI); gloo works for CPU tests of the same code.

Partitioning: a global step is G consecutive batches of the reference's single
numpy stream; rank r assembles batch r and *replays* (consumes without building) the others, so
the union of the ranks' batches is exactly what a single process would train on G steps.  A
64-graph batch never splits across GPUs (attention couples all graphs of a batch).

Supervised step: the only collective is the gradient all-reduce (average) over the flat fp32
gradient buffer, issued in a few large buckets: xGMI is point-to-point (7 links per GPU), so RCCL's
ring/tree bandwidth per collective is what matters, and a handful of multi-MB buckets keeps it
link-bound rather than latency-bound.  Clip + Adam then run redundantly (bit-identically) on every rank.

Unsupervised step (UnSupGradSync): the encoder gradients (37 K floats at C5) are all-reduced; the
embedding table's gradient (ss.weight, [V, D] = 10.2 M floats at C5) is non-zero only on the rows a
batch touches -- its nodes' labels and the 512 sampled ids (sampled_softmax.py:45,48) -- so those rows
are all-gathered (ids + values, ~40 KB per rank at C5) and folded into every rank's dense gradient
in rank order: the dense all-reduce's result at a fraction of its bytes.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch


def _avg_op(dist, group):
    """ReduceOp.AVG where it pays: RCCL with more than one rank (ncclAvg pre-multiplies 1/world inside the ring
    reduction, so no separate scaling pass over the gradient buffer), else None -- SUM and the callers scale by
    1/world only when world > 1.  (At one rank SUM in place launches nothing while AVG runs RCCL's one-rank
    pre-multiply kernel over every bucket: 5 x 14 us per C4 step, profiles/r06/dp_overhead_ab.txt.)"""
    try:
        return dist.ReduceOp.AVG if dist.get_backend(group) == "nccl" and dist.get_world_size(group) > 1 else None
    except (RuntimeError, ValueError):
        return None


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
        self.avg = _avg_op(dist, group)

    def __call__(self, flat) -> None:
        g = flat.gflat
        handles = []
        op = self.avg if self.avg is not None else self.dist.ReduceOp.SUM
        for o in range(0, g.numel(), self.bucket):
            handles.append(self.dist.all_reduce(g[o:o + self.bucket], op=op, group=self.group, async_op=True))
        for h in handles:
            h.wait()
        if self.avg is None and self.world > 1:
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

    RCCL at world > 1: ncclAvg (the 1/world folded into the ring reduction) instead of the scaling pass.  (Measured
    and not kept, round 6: the collectives issued straight to torch's librccl through ctypes on the gradients' own
    stream, no c10d events -- 4.82 vs 3.36 ms per C4 step at one rank, the host blocked ~190 us in each call;
    profiles/r06/dp_overhead_ab.txt.)
    """

    def __init__(self, flat, group=None, bucket_mb: float = 4.0, layer_prefix: str = "u2gnn_layers."):
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
        # Adjacent layer regions go out together until a bucket holds >= bucket_mb; the backward visits the layers in
        # descending flat order, so each new region ends where the bucket begins.  The parameters after the last
        # layer (the head, written before the encoder backward starts) join the first bucket.  Default 4 MB: every
        # C4 layer (5.2 MB) its own collective -- at one rank 2 buckets of 2 layers measured the same as 5
        # collectives (+74 vs +72-85 us over no process group, profiles/r06/dp_overhead_ab.txt), and at N ranks a
        # smaller last bucket is less exposed after the backward.
        self.bucket = max(1, int(bucket_mb * (1 << 20) // 4))
        layers = {n[:n.index(".layers.") + len(".layers.")] + n.split(".layers.")[1].split(".")[0]
                  for n in flat.names if n.startswith(layer_prefix) and ".layers." in n}
        self.n_layers = len(layers)
        enc_hi = max((b for n, (a, b) in self.span.items() if n.startswith(layer_prefix)), default=0)
        self.tail = (self._align_end(enc_hi), flat.gflat.numel())   # [head parameters, end)
        self.acc: Optional[Tuple[int, int]] = None
        self.acc_stream = None
        self.calls = 0
        # RCCL: the average inside the collective (ncclAvg) -- no scaling pass over the 20.7 MB buffer at the
        # step's end; gloo: sum, then the scaling pass
        self.avg = _avg_op(dist, group)
        self.op = self.avg if self.avg is not None else dist.ReduceOp.SUM


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

    def _issue(self, lo: int, hi: int, stream) -> None:
        g = self.flat.gflat
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            self.pending.append(self.dist.all_reduce(g[lo:hi], op=self.op, group=self.group, async_op=True))
        self.launched.append((lo, hi))

    def layer_done(self, prefix: str, stream: Optional["torch.cuda.Stream"] = None) -> None:
        lo, hi = self.region(prefix)
        self.calls += 1
        if self.acc is None and self.calls == 1 and hi == self.tail[0] and self.tail[1] > self.tail[0]:
            hi = self.tail[1]   # the head's gradients: complete before the encoder backward, adjacent
        if self.acc is not None and hi != self.acc[0]:   # not adjacent: send what is held
            self._issue(*self.acc, self.acc_stream)
            self.acc = None
        self.acc = (lo, self.acc[1] if self.acc is not None else hi)
        self.acc_stream = stream   # ordered after every earlier write (the side stream forks from the main one)
        if self.acc[1] - self.acc[0] >= self.bucket or self.calls >= self.n_layers:
            self._issue(*self.acc, self.acc_stream)
            self.acc = None

    def __call__(self, flat) -> None:
        g = flat.gflat
        if self.acc is not None:   # (a backward that visited fewer layers than the stack holds)
            self._issue(*self.acc, self.acc_stream)
            self.acc = None
        self.calls = 0
        o = 0
        for lo, hi in sorted(self.launched) + [(g.numel(), g.numel())]:
            if lo > o:   # a region no layer_done covered (head parameters, padding)
                self.pending.append(self.dist.all_reduce(g[o:lo], op=self.op, group=self.group, async_op=True))
            o = max(o, hi)
        for h in self.pending:
            h.wait()
        self.pending.clear()
        self.launched.clear()
        if self.avg is None and self.world > 1:
            g.mul_(1.0 / self.world)


def broadcast_params(flat, src: int = 0, group=None) -> None:
    import torch.distributed as dist
    dist.broadcast(flat.flat, src, group=group)


def max_batch_nodes(node_start, batch_size: int) -> int:
    """An upper bound on the nodes of any batch of `batch_size` graphs (the sum of the largest graph
    sizes): the fixed per-rank row count of the label-row all-gather, so that no rank has to learn
    the others' batch sizes (no host synchronisation inside a step)."""
    sizes = np.diff(np.asarray(node_start, dtype=np.int64))
    return int(np.sort(sizes)[::-1][:batch_size].sum())


class UnSupGradSync:
    """Data-parallel gradient exchange of the unsupervised U2GNN step (SURVEY.md §8(e);
    train_pytorch_U2GNN_UnSup.py:149-162).  Rank r trains batch r of each group of `world` consecutive
    batches (rank_batches) with the r-th sample draw of the group, so the ranks together see exactly
    what one process sees in `world` steps; the averaged gradient is their mean.

    * ``__call__(flat)``: all-reduce (sum, then 1/world) of the encoder region of the flat gradient;
      the ss.weight region is excluded (its rows come from ``rows``).
    * ``buffers(n_lab, n_smp, D, device)``: the compact-row views the sampled-softmax backward writes into
      directly (u2gnn_sampled_softmax_bwd_rows): each lives in ONE flat exchange buffer per kind that holds
      the row ids (int64, as pairs of floats) followed by the rows, so a kind crosses the ranks in one
      all-gather.
    * ``rows(ids_lab, rows_lab, ids_smp, rows_smp, gW)``: all-gather every rank's compact rows (label rows
      padded with id -1 to ``id_cap``; the S sample rows) and fold them into the dense gW (all zero on
      entry) in rank order, labels before samples, scaled by 1/world -- the same destinations in the same
      order on every rank, so every rank holds the same bits.  Returns the gathered id tensors (the rows
      to zero after the optimizer step).  Rows not written in the ``buffers`` views are copied in.

    Device tensors go through u2gnn_index_add_rows (id -1 rows skipped); CPU tensors (the gloo tests)
    through torch's index_add_ with the padding rows dropped -- the same sums in the same order."""

    def __init__(self, flat, id_cap: int, group=None, weight_name: str = "ss.weight"):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        g = flat.grads[weight_name]
        self.lo = (g.data_ptr() - flat.gflat.data_ptr()) // 4
        self.hi = self.lo + g.numel()
        self.id_cap = int(id_cap)
        self._bufs: Dict = {}

    def __call__(self, flat) -> None:
        g = flat.gflat
        regions = [(0, self.lo), (self.hi, g.numel())]
        avg = _avg_op(self.dist, self.group)
        for a, b in regions:
            if b > a:
                self.dist.all_reduce(g[a:b], op=avg if avg is not None else self.dist.ReduceOp.SUM, group=self.group)
                if avg is None and self.world > 1:
                    g[a:b].mul_(1.0 / self.world)

    def _flat(self, kind: str, rows: int, D: int, device) -> torch.Tensor:
        """[2 * rows + rows * D] float32: the ids (int64 bits) then the rows, one all-gather per kind."""
        key = (kind, rows, D, str(device))
        buf = self._bufs.get(key)
        if buf is None:
            n = 2 * rows + rows * D
            n += n & 1   # even length: every rank's chunk of the gathered buffer starts 8-byte aligned (int64 ids)
            buf = self._bufs[key] = torch.zeros(n, dtype=torch.float32, device=device)
            buf[:2 * rows].view(torch.int64).fill_(-1)
            if kind == "lab":
                self._bufs[("neg", str(device))] = torch.full((rows,), -1, dtype=torch.int64, device=device)
        return buf

    def buffers(self, n_lab: int, n_smp: int, D: int, device):
        if n_lab > self.id_cap:
            raise ValueError(f"batch has {n_lab} label rows, above the exchange cap {self.id_cap}")
        lab = self._flat("lab", self.id_cap, D, device)
        smp = self._flat("smp", n_smp, D, device)
        cap = self.id_cap
        return (lab[2 * cap:2 * cap + cap * D].view(cap, D)[:n_lab], smp[2 * n_smp:2 * n_smp + n_smp * D].view(n_smp, D))

    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        # concatenated along dim 0 (the layout both RCCL and gloo accept), viewed as [world, ...]
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
        self.dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out.view((self.world,) + tuple(t.shape))

    def rows(self, ids_lab: torch.Tensor, rows_lab: torch.Tensor, ids_smp: torch.Tensor, rows_smp: torch.Tensor,
             gW: torch.Tensor):
        n, D = rows_lab.shape
        S = rows_smp.shape[0]
        cap = self.id_cap
        rl, _ = self.buffers(n, S, D, rows_lab.device)
        bsmp = self._flat("smp", S, D, rows_lab.device)
        if rows_lab.data_ptr() != rl.data_ptr():
            rl.copy_(rows_lab)
        if rows_smp.data_ptr() != bsmp[2 * S:].data_ptr():
            bsmp[2 * S:2 * S + S * D].view(S, D).copy_(rows_smp)
        lab = self._flat("lab", cap, D, rows_lab.device)
        neg = self._bufs[("neg", str(rows_lab.device))]
        torch.cat([ids_lab.to(torch.int64), neg[:cap - n]], out=lab[:2 * cap].view(torch.int64))
        bsmp[:2 * S].view(torch.int64).copy_(ids_smp)
        g_lab, g_smp = self._gather(lab), self._gather(bsmp)
        alpha = 1.0 / self.world
        ids_l, ids_s = [], []
        for r in range(self.world):
            il, rr = g_lab[r, :2 * cap].view(torch.int64), g_lab[r, 2 * cap:2 * cap + cap * D].view(cap, D)
            is_, rs = g_smp[r, :2 * S].view(torch.int64), g_smp[r, 2 * S:2 * S + S * D].view(S, D)
            _index_add(gW, il, rr, alpha)
            _index_add(gW, is_, rs, alpha)
            ids_l.append(il)
            ids_s.append(is_)
        return (torch.cat(ids_l), torch.cat(ids_s))


def _index_add(dst: torch.Tensor, ids: torch.Tensor, rows: torch.Tensor, alpha: float) -> None:
    if dst.is_cuda:
        from . import kernels as K
        K.index_add_rows(rows, ids, dst, alpha)
    else:   # gloo tests on CPU: the same per-element sum dst += alpha * row
        keep = ids >= 0
        dst.index_add_(0, ids[keep], rows[keep] * alpha)
