"""Fused training steps (no autograd, no host sync inside a step).

``SupTrainer.step`` = one iteration of train() in train_pytorch_U2GNN_Sup.py:152-162:
label_smoothing + soft cross-entropy, backward, clip_grad_norm_(0.5), Adam.step() — on the
HIP kernels, with gradients written straight into the flat grad buffer.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import kernels as K
from .core import DeviceBatch, FusedAdam


class SupTrainer:
    def __init__(self, model, lr: float, max_norm: Optional[float] = 0.5, seed: int = 123):
        self.m = model
        self.flat = model.flatten_parameters()
        self.opt = FusedAdam(self.flat, lr, max_norm)
        dev = self.flat.flat.device
        self.loss = torch.zeros(1, device=dev)
        self.gen = torch.Generator().manual_seed(seed)
        self.grad_sync = None   # optional callable(flat) for data-parallel all-reduce

    def next_seed(self) -> int:
        return int(torch.randint(0, 2 ** 62, (1,), generator=self.gen).item())

    def forward_backward(self, b: DeviceBatch, train: bool = True, seed: Optional[int] = None) -> torch.Tensor:
        """seed: the step's dropout seed (default: the trainer's own generator; the data-parallel CLIs pass
        the batch's stream-position seed, u2gnn_hip.cli.step_seed)."""
        core = self.m.core
        scores, ctx = core.forward(b, train, need_ctx=True, seed=self.next_seed() if seed is None else int(seed))
        dscores = torch.empty_like(scores)
        K.smoothed_ce(scores, b.labels, b.B, core.C, 0.1, self.loss, dscores)
        core.backward(ctx, dscores, self.flat.grads)
        return self.loss

    def step(self, b: DeviceBatch, train: bool = True, seed: Optional[int] = None) -> torch.Tensor:
        loss = self.forward_backward(b, train, seed)
        if self.grad_sync is not None:
            self.grad_sync(self.flat)
        self.opt.step()
        return loss

    def set_lr(self, lr: float):
        self.opt.set_lr(lr)


class StepGraphs:
    """HIP-graph replay of a trainer's step (SupTrainer.step(b) / UnSupTrainer.step(b, sample_ids)).

    The first step with a given set of argument objects is captured into a torch.cuda.CUDAGraph
    (the capture stream plus the parameter-gradient side stream, joined through events) and every
    step with them afterwards is ONE graph launch instead of ~180 host-issued kernels — the
    latency-bound d = 4 UnSup step (C5) is host-bound otherwise.  One graph per distinct batch
    (shapes differ); each keeps its own private memory pool.  What changes from step to step lives
    in HBM and is advanced by the graph's first node (u2gnn_step_advance): the seed epoch that every
    dropout-drawing kernel mixes into its capture-time seed (u2gnn_set_seed_epoch) and Adam's step
    count (FusedAdam.use_device_schedule), so replays draw fresh masks and follow torch's Adam
    schedule exactly as the eager step does."""

    def __init__(self, trainer):
        self.tr = trainer
        dev = trainer.flat.flat.device
        self.epoch = torch.zeros(1, device=dev, dtype=torch.int64)
        K.set_seed_epoch(self.epoch)
        trainer.opt.use_device_schedule()
        # key -> (graph, the argument objects it was captured with).  The graph holds their device
        # pointers and shapes, so the objects are kept alive here: a freed batch whose id() is reused
        # by a new object would otherwise replay a graph over freed memory.
        self.graphs = {}
        self._open = True

    def capture(self, *args) -> "torch.cuda.CUDAGraph":
        if not self._open:
            raise RuntimeError("StepGraphs is closed")
        key = tuple(id(a) for a in args)
        ent = self.graphs.get(key)
        if ent is None:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                # the step's first launch (the weight pack) bumps the epoch and Adam's t before anything else
                # runs (u2gnn_pack_padded_multi_adv): one launch less than a u2gnn_step_advance node
                K.defer_step_advance(self.epoch, self.tr.opt.t_dev)
                try:
                    self.tr.step(*args)
                finally:
                    pending = K.step_advance_pending()
                    K._PENDING_ADVANCE.clear()
                if pending:
                    raise RuntimeError("StepGraphs: the captured step ran no weight pack to carry the step advance")
            ent = self.graphs[key] = (g, args)
        return ent[0]

    def step(self, *args) -> torch.Tensor:
        self.capture(*args).replay()
        return self.tr.loss

    def close(self) -> None:
        """Back to eager steps: the epoch pointer is released, Adam's step count returns to the host.
        Idempotent; also run by the context manager and the finaliser, so the process-wide epoch
        pointer never outlives self.epoch."""
        if not self._open:
            return
        self._open = False
        torch.cuda.synchronize()
        K.set_seed_epoch(None)
        self.tr.opt.use_host_schedule()
        self.graphs.clear()

    def __enter__(self) -> "StepGraphs":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown: the library may already be gone
            pass
