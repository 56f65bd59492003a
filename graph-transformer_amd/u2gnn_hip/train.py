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

    def forward_backward(self, b: DeviceBatch, train: bool = True) -> torch.Tensor:
        core = self.m.core
        scores, ctx = core.forward(b, train, need_ctx=True, seed=self.next_seed())
        dscores = torch.empty_like(scores)
        K.smoothed_ce(scores, b.labels, b.B, core.C, 0.1, self.loss, dscores)
        core.backward(ctx, dscores, self.flat.grads)
        return self.loss

    def step(self, b: DeviceBatch, train: bool = True) -> torch.Tensor:
        loss = self.forward_backward(b, train)
        if self.grad_sync is not None:
            self.grad_sync(self.flat)
        self.opt.step()
        return loss

    def set_lr(self, lr: float):
        self.opt.lr = lr
