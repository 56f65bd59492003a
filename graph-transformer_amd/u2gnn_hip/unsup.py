"""Unsupervised U2GNN on the gfx950 kernels.

Working semantics of the fork's UnSup model (the shipped file cannot run):
per-U2GNN-layer slot-0 outputs concatenated to [N, d*L] (pytorch_U2GNN_UnSup.py:52-69,
U2GNN_tf/model_U2GNN_Unsup_multi.py:43-55) -> dropout (:56 of the TF model) -> SampledSoftmax
over the node vocabulary with 512 log-uniform samples (sampled_softmax.py:36-56); the training
loss is the SUM of the per-node losses (train_pytorch_U2GNN_UnSup.py:156).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import kernels as K
from .core import DeviceBatch, EncoderStack, FlatParams, FusedAdam
from .engine import rup, site_seed

SITE_SS_DROP = 6


class UnSupCore:
    def __init__(self, module, precision: str = "fp32"):
        self.m = module
        self.d = module.feature_dim_size
        self.ff = module.ff_hidden_size
        self.L = module.num_U2GNN_layers
        self.T = module.num_self_att_layers
        self.p_out = module.dropout_p
        self.stack = EncoderStack(module.u2gnn_layers, self.d, self.ff, self.T, self.L, precision, 0.5,
                                  getattr(module, "attention", "nodes"))

    def encode(self, b: DeviceBatch, train: bool, need_ctx: bool, seed: int, p: float = 0.0, drop_seed: int = 0):
        """-> (OV f32 [N, d*L] real layout, dropped out with (p, drop_seed) when p > 0, ctx).  The padded
        per-layer outputs are unpadded, concatenated and dropped out in one launch (u2gnn_concat_dropout)."""
        outs, sctx = self.stack.forward(b, train, need_ctx, seed)
        d, dp, L = self.d, rup(self.d, 64), self.L
        N = b.N
        OV = torch.empty(N, d * L, device=b.X_concat.device, dtype=torch.float32)
        K.concat_dropout(outs, dp, N, d, OV, d * L, p, drop_seed)
        return OV, sctx

    def encode_backward(self, sctx, dOV: torch.Tensor, grads: dict, p: float = 0.0, drop_seed: int = 0):
        """dOV: the gradient of encode()'s output; its dropout (same p, drop_seed) and the split into the
        layers' padded gradients are one launch (u2gnn_split_dropout_bwd)."""
        d, dp, L = self.d, rup(self.d, 64), self.L
        dims = sctx["dims"]
        dXs = [torch.empty(dims.Np, dp, device=dOV.device, dtype=torch.float32) for _ in range(L)]
        K.split_dropout_bwd(dOV, d * L, dims.N, dims.Np, d, dp, p, drop_seed, dXs)
        return self.stack.backward(sctx, lambda l: dXs[l], grads)


class UnSupTrainer:
    """One iteration of train() in train_pytorch_U2GNN_UnSup.py:152-160, fused on device:
    encode -> dropout -> sampled softmax (sum loss) -> backward -> clip(0.5) -> Adam (dense over
    the whole embedding table, like torch.optim.Adam on a dense gradient)."""

    def __init__(self, model, lr: float, max_norm: Optional[float] = 0.5, seed: int = 123):
        self.m = model
        self.core: UnSupCore = model.core
        self.flat = FlatParams(model, names=model.trainable_names())
        self.opt = FusedAdam(self.flat, lr, max_norm)
        dev = self.flat.flat.device
        self.loss = torch.zeros(1, device=dev)
        self.ws = torch.empty(1024, device=dev)
        self.gen = torch.Generator().manual_seed(seed)
        # data parallelism (dp.UnSupGradSync): grad_sync(flat) averages the encoder gradients,
        # row_sync.rows(...) exchanges the touched rows of ss.weight's gradient
        self.grad_sync = None
        self.row_sync = None
        # ss.weight rows written by this step's gradient (zeroed again after the optimizer step)
        self._touched = ()
        # tests: keep the last step's encoder context (saved activations) as self.last_ctx
        self.keep_ctx = False
        self.last_ctx = None

    def next_seed(self) -> int:
        return int(torch.randint(0, 2 ** 62, (1,), generator=self.gen).item())

    def forward_backward(self, b: DeviceBatch, sample_ids: torch.Tensor, train: bool = True,
                         seed: Optional[int] = None):
        core, ss = self.core, self.m.ss
        # the dense ss.weight gradient must be all zero on entry (the backward adds rows into it): rows a
        # previous forward_backward wrote and no step()/clear_row_grads() zeroed (an evaluation loss, a
        # gradient check, an exception between backward and step) are zeroed first
        if self._touched:
            self.clear_row_grads()
        seed = self.next_seed() if seed is None else int(seed)
        p = core.p_out if train else 0.0
        ds = site_seed(seed, 0, 0, SITE_SS_DROP)
        OVd, sctx = core.encode(b, train, True, seed, p, ds)   # dropout fused into the concatenation
        if self.keep_ctx:
            self.last_ctx = sctx
        N, D = OVd.shape
        W = ss.weight
        S = sample_ids.numel()
        lrow = torch.empty(N, device=OVd.device)
        prob = torch.empty(N, S, device=OVd.device)
        K.sampled_softmax_fwd(OVd, D, b.input_y, sample_ids, S, W, W.stride(0), lrow, prob, N, D)
        K.sum_all(lrow, N, self.loss)
        self.last_logits = lrow   # per-node losses of the step (the reference forward's output)
        # W's gradient touches only the label rows and the S sampled rows (sampled_softmax.py:45,48):
        # the backward writes them as compact rows, folded into the dense gradient (all zero between
        # steps, so no dense zero fill of the [V, D] table) -- locally, or after the data-parallel
        # row exchange
        gW = self.flat.grads["ss.weight"]
        dOV = torch.empty_like(OVd)
        if self.row_sync is not None:   # data parallel: compact rows, exchanged before they are added
            # written straight into the exchange buffers (ids + rows of one kind cross the ranks together)
            rows_lab, rows_smp = self.row_sync.buffers(N, S, D, OVd.device)
            K.sampled_softmax_bwd_rows(OVd, D, b.input_y, sample_ids, S, W, W.stride(0), prob, None, dOV, D,
                                       rows_lab, rows_smp, N, D)
            self._touched = self.row_sync.rows(b.input_y, rows_lab, sample_ids, rows_smp, gW)
        else:
            # added straight into the dense gradient, labels (one kernel) before samples (the next): the
            # destinations within each kernel are distinct, so this is the compact-rows form followed by
            # its two index_add launches, value for value, in two launches instead of four
            K.sampled_softmax_bwd(OVd, D, b.input_y, sample_ids, S, W, W.stride(0), prob, None, dOV, D, gW,
                                  gW.stride(0), N, D)
            self._touched = (b.input_y, sample_ids)
        core.encode_backward(sctx, dOV, self.flat.grads, p, ds)   # dropout's backward fused into the split
        return self.loss

    def step(self, b: DeviceBatch, sample_ids: torch.Tensor, train: bool = True, seed: Optional[int] = None):
        loss = self.forward_backward(b, sample_ids, train, seed)
        if self.grad_sync is not None:
            self.grad_sync(self.flat)
        self.opt.step()
        self.clear_row_grads()
        return loss

    def clear_row_grads(self):
        """Zero the ss.weight gradient rows this step wrote (the dense gradient is all zero between
        steps; torch's Adam sees the same dense gradient either way)."""
        gW = self.flat.grads["ss.weight"]
        if len(self._touched) == 2:   # labels and samples: one launch
            K.index_zero_rows2(self._touched[0], self._touched[1], gW)
        else:
            for ids in self._touched:
                K.index_zero_rows(ids, gW)
        self._touched = ()


def graph_embeddings(weight: torch.Tensor, node_start: np.ndarray) -> torch.Tensor:
    """evaluate() of train_pytorch_U2GNN_UnSup.py:167-169: spmm(graph_pool, ss.weight), i.e. the
    per-graph sum of the learned node embeddings (graph_pool over ALL graphs, nodes contiguous)."""
    dev = weight.device
    G = len(node_start) - 1
    V, D = weight.shape
    out = torch.empty(G, D, device=dev)
    rowptr = torch.as_tensor(np.asarray(node_start), dtype=torch.int64, device=dev)
    col = torch.arange(V, device=dev, dtype=torch.int64)
    vals = torch.ones(V, device=dev)
    K.pool_fwd(weight, D, rowptr, col, vals, out, D, G, D, 0.0, 0)
    return out


def fold_accuracies(emb: np.ndarray, labels: np.ndarray, splits) -> list:
    """The classifier half of evaluate() (train_pytorch_U2GNN_UnSup.py:171-181): per (train, test) split
    a LogisticRegression(solver="liblinear", tol=0.001) on the graph embeddings; returns the test
    accuracies.  Host code (sklearn), after graph_embeddings on the device."""
    from sklearn.linear_model import LogisticRegression
    accs = []
    for train_idx, test_idx in splits:
        cls = LogisticRegression(solver="liblinear", tol=0.001)
        cls.fit(emb[train_idx], labels[train_idx])
        accs.append(float(cls.score(emb[test_idx], labels[test_idx])))
    return accs
