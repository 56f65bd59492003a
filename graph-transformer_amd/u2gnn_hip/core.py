"""Model-level orchestration of the U2GNN hot path on the gfx950 kernels.

* ``DeviceBatch``   — one mini-batch resident in HBM (input_x, X_concat, pooling CSR, labels).
* ``SupCore``       — forward / backward of pytorch_U2GNN_Sup.TransformerU2GNN (:30-46):
                      gather -> L x (T encoder layers -> sum-pool -> dropout -> Linear, summed).
* ``FlatParams``    — all parameters (and grads, Adam moments) in single flat fp32 buffers,
                      so clip_grad_norm_ + Adam are two sweeps (train_pytorch_U2GNN_Sup.py:160-161).
* ``FusedAdam``     — torch.optim.Adam semantics with the clip coefficient applied on device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import kernels as K
from . import native
from .engine import deep_wgrad as engine_deep_wgrad
from .engine import (SITE_ATTN, SITE_DROP1, SITE_DROP2, SITE_DROPFF, SITE_HEAD, Dims, LayerParams, PackedLayer,
                     OffPath, encoder_layer_backward, encoder_layer_forward, rup, side_stream_pays, site_seed)


_IOTA = {}


_COPY: dict = {}


def _copy_stream(dev: torch.device) -> "torch.cuda.Stream":
    s = _COPY.get(dev.index)
    if s is None:
        s = _COPY[dev.index] = torch.cuda.Stream(device=dev)
    return s


def _pool_iota(N: int, dev: torch.device):
    """graph_pool's column indices (0..N-1) and values (ones) as views of cached device buffers."""
    key = (dev.type, dev.index)
    c = _IOTA.get(key)
    if c is None or c[0].numel() < N:
        n = max(N, 1 << 14, 2 * (c[0].numel() if c is not None else 0))
        c = _IOTA[key] = (torch.arange(n, device=dev, dtype=torch.int64), torch.ones(n, device=dev, dtype=torch.float32))
    return c[0][:N], c[1][:N]


@dataclass
class DeviceBatch:
    N: int
    B: int
    input_x: torch.Tensor           # int64 [N, k+1] (only column 0 is read: the slot-0 gather)
    X_concat: torch.Tensor          # f32 [N, d]
    rowptr: torch.Tensor            # int64 [B+1]   pooling CSR (graph_pool rows)
    colidx: torch.Tensor            # int64 [nnz]
    vals: torch.Tensor              # f32 [nnz]
    labels: Optional[torch.Tensor] = None   # int64 [B]
    input_y: Optional[torch.Tensor] = None  # int64 [N] (UnSup softmax labels)
    # int32[1] device flag the gather / scatter kernels set on an out-of-range input_x entry (they
    # read and write nothing there); the constructors validate input_x up front, so it stays 0
    err: Optional[torch.Tensor] = None
    # True when colidx is 0..N-1 in order (batches built from offsets, _pool_iota): the pool backward
    # then stores every row of its output (u2gnn_pool_bwd_rows) instead of accumulating into zeros
    block_rows: bool = False

    def __post_init__(self):
        if self.err is None:
            self.err = torch.zeros(1, device=self.X_concat.device, dtype=torch.int32)

    def check_indices(self):
        """IndexError if a kernel met an out-of-range input_x entry (host sync; F.embedding raises)."""
        if int(self.err.item()):
            raise IndexError("index out of range in self (input_x entry outside [0, N))")

    @property
    def idx_stride(self):
        return self.input_x.stride(0)

    @staticmethod
    def from_offsets(input_x, offsets, X_concat, labels=None, device="cuda", input_y=None):
        """Host arrays (numpy / torch CPU) -> HBM.  Block-diagonal graph_pool of ones given by
        node offsets (train_pytorch_U2GNN_Sup.py:73-89)."""
        dev = torch.device(device)
        _check_range_host(input_x, int(np.asarray(offsets)[-1]))
        ix = torch.as_tensor(input_x, dtype=torch.int64).to(dev, non_blocking=True).contiguous()
        X = torch.as_tensor(X_concat, dtype=torch.float32).to(dev, non_blocking=True).contiguous()
        off = torch.as_tensor(np.asarray(offsets), dtype=torch.int64)
        N = int(off[-1])
        B = off.numel() - 1
        lab = None if labels is None else torch.as_tensor(labels, dtype=torch.int64).to(dev, non_blocking=True)
        iy = None if input_y is None else torch.as_tensor(input_y, dtype=torch.int64).to(dev, non_blocking=True)
        return DeviceBatch(N, B, ix, X, off.to(dev), torch.arange(N, device=dev, dtype=torch.int64),
                           torch.ones(N, device=dev, dtype=torch.float32), lab, iy, block_rows=True)

    @staticmethod
    def from_store(hb, X_dev: torch.Tensor, device="cuda"):
        """A natively assembled batch (GraphStore.assemble(..., gather_x=False)) -> HBM: input_x, offsets
        and the rows' dataset node ids cross PCIe asynchronously from page-locked buffers (~0.7 MB at
        C4 instead of the 7 MB X_concat; BatchLoader assembles straight into a ring of them);
        X_concat is gathered on the GPU from the dataset's device-resident features X_dev [V, d]
        (u2gnn_gather_rows).  No host synchronisation."""
        from . import kernels as K
        dev = torch.device(device)
        N, B = int(hb.offsets[-1]), len(hb.offsets) - 1
        slot = getattr(hb, "pinned", None)
        _check_range_host(hb.input_x, N)
        if slot is not None and dev.type == "cuda":
            # the batch's transfers and its feature gather run on a copy stream, so the next batch
            # crosses PCIe while the current step computes; the compute stream waits on one event
            main = torch.cuda.current_stream(dev)
            cs = _copy_stream(dev)
            k1 = hb.input_x.shape[1]
            with torch.cuda.stream(cs):
                h2d = lambda t: t.to(dev, non_blocking=True)  # noqa: E731
                ix = h2d(slot.ix[:N * k1]).view(N, k1)
                gnode, off, lab = h2d(slot.gnode[:N]), h2d(slot.offsets[:B + 1]), h2d(slot.labels[:B])
                slot.event = torch.cuda.Event()
                slot.event.record()
                d = X_dev.shape[1]
                X = torch.empty(N, d, device=dev, dtype=torch.float32)
                if N:
                    K.gather_rows(X_dev, gnode, 1, X, N, N, d, d)
                err = torch.zeros(1, device=dev, dtype=torch.int32)
            ready = torch.cuda.Event()
            ready.record(cs)
            main.wait_event(ready)
            for t in (ix, gnode, off, lab, X, err):   # allocated on the copy stream, used on the compute one
                t.record_stream(main)
            iy = gnode if hb.input_y is not None else None
            colidx, vals = _pool_iota(N, dev)
            return DeviceBatch(N, B, ix, X, off, colidx, vals, lab, iy, err, block_rows=True)
        if slot is not None:
            k1 = hb.input_x.shape[1]
            h2d = lambda t: t.to(dev, non_blocking=True)  # noqa: E731
            ix = h2d(slot.ix[:N * k1]).view(N, k1)
            gnode, off, lab = h2d(slot.gnode[:N]), h2d(slot.offsets[:B + 1]), h2d(slot.labels[:B])
            slot.event = torch.cuda.Event()
            slot.event.record()
            iy = gnode if hb.input_y is not None else None   # UnSup labels = dataset node ids
        else:
            pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(dev, non_blocking=True)  # noqa: E731
            ix, gnode, off = pin(hb.input_x), pin(hb.gnode), pin(np.asarray(hb.offsets, dtype=np.int64))
            lab = None if hb.labels is None else pin(np.asarray(hb.labels, dtype=np.int64))
            iy = None if hb.input_y is None else pin(np.asarray(hb.input_y, dtype=np.int64))
        d = X_dev.shape[1]
        X = torch.empty(N, d, device=dev, dtype=torch.float32)
        if N:
            K.gather_rows(X_dev, gnode, 1, X, N, N, d, d)
        colidx, vals = _pool_iota(N, dev)
        return DeviceBatch(N, B, ix, X, off, colidx, vals, lab, iy, block_rows=True)

    @staticmethod
    def from_reference_inputs(input_x, graph_pool, X_concat, labels=None):
        """The reference forward() inputs: input_x int64 [N,k+1], graph_pool sparse COO [B,N],
        X_concat f32 [N,d] (pytorch_U2GNN_Sup.py:30)."""
        dev = X_concat.device
        gp = graph_pool.coalesce()
        B, N = gp.shape
        if input_x.numel() and (int(input_x.min()) < 0 or int(input_x.max()) >= int(N)):
            raise IndexError("index out of range in self (input_x entry outside [0, N))")
        rows, cols = gp.indices()
        vals = gp.values().to(torch.float32)
        rowptr = torch.zeros(B + 1, dtype=torch.int64, device=dev)
        rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=B), 0)
        return DeviceBatch(int(N), int(B), input_x.to(dev).contiguous(), X_concat.to(torch.float32).contiguous(),
                           rowptr, cols.contiguous(), vals.contiguous(), labels)


def _check_range_host(input_x, N: int):
    """F.embedding(input_x, X_concat) raises IndexError for an entry outside [0, N) (pytorch_U2GNN_Sup.py:32)."""
    a = input_x.numpy() if isinstance(input_x, torch.Tensor) else np.asarray(input_x)
    if a.size and (int(a.min()) < 0 or int(a.max()) >= N):
        raise IndexError("index out of range in self (input_x entry outside [0, N))")


class EncoderStack:
    """L U2GNN layers x T post-LN encoder layers on slot-0 rows, with the re-gather between
    U2GNN layers (pytorch_U2GNN_Sup.py:33-39; pytorch_U2GNN_UnSup.py:55-64)."""

    def __init__(self, u2gnn_layers, d: int, ff: int, T: int, L: int, prec: str = "fp32", p_enc: float = 0.5,
                 attention: str = "nodes"):
        self.layers, self.d, self.ff, self.T, self.L, self.prec, self.p_enc = u2gnn_layers, d, ff, T, L, prec, p_enc
        if attention not in ("nodes", "neighbors"):
            raise ValueError(f"attention must be 'nodes' or 'neighbors', got {attention!r}")
        self.attention = attention
        self.packed = None
        # optional callable(prefix, stream): called once a layer's parameter gradients are
        # enqueued (on `stream`), e.g. dp.OverlappedGradAllReduce.layer_done
        self.grad_ready = None

    def layer_params(self, l, t) -> LayerParams:
        return LayerParams.from_encoder_layer(self.layers[l].layers[t])

    def _pack(self, device):
        if self.packed is None:
            self.packed = [[PackedLayer(self.d, self.ff, device) for _ in range(self.T)] for _ in range(self.L)]
        jobs = []
        for l in range(self.L):
            for t in range(self.T):
                jobs += self.packed[l][t].jobs(self.layer_params(l, t))
        K.pack_padded_multi(jobs)      # one launch per 32 tensors

    def forward(self, b: "DeviceBatch", train: bool, need_ctx: bool, seed: int):
        """Returns (outs, ctx): outs[l] = padded [Np, dp] slot-0 output of U2GNN layer l."""
        if self.attention == "neighbors":
            return self._forward_neighbors(b, train, need_ctx, seed)
        dev = b.X_concat.device
        d, dp = self.d, rup(self.d, 64)
        dims = Dims(b.N, d, self.ff)
        Np = dims.Np
        self._pack(dev)
        X = torch.empty(Np, dp, device=dev, dtype=torch.float32)
        K.gather_rows(b.X_concat, b.input_x, b.idx_stride, X, b.N, Np, d, dp, b.err)
        outs, lctxs = [], []
        for l in range(self.L):
            lctx = []
            for t in range(self.T):
                seeds = {s: site_seed(seed, l, t, s) for s in (SITE_ATTN, SITE_DROP1, SITE_DROPFF, SITE_DROP2)}
                if native.enabled():
                    X, c = native.layer_forward(X, self.packed[l][t], self.layer_params(l, t), dims, train, seeds,
                                                need_ctx, self.prec, self.p_enc, deep_wgrad=engine_deep_wgrad())
                else:
                    X, c = encoder_layer_forward(X, self.packed[l][t], self.layer_params(l, t), dims, train, seeds,
                                                 need_ctx, self.prec, self.p_enc)
                lctx.append(c)
            outs.append(X)
            lctxs.append(lctx)
            if l + 1 < self.L:
                Xn = torch.empty(Np, dp, device=dev, dtype=torch.float32)
                K.gather_rows(X, b.input_x, b.idx_stride, Xn, b.N, Np, d, dp, b.err)
                X = Xn
        return outs, {"dims": dims, "layers": lctxs, "batch": b}

    # ---- paper semantics (U2GNN_tf/model_U2GNN_Sup_multi.py:14-45): every
    # node attends over its own k+1 gathered neighbour tokens.  Token rows are node-major
    # (row n*W + s = slot s of node n, W = k+1); each layer runs on all N*W tokens through the native
    # executor's window mode; slot 0 of the last layer is the node's output.
    def _forward_neighbors(self, b: "DeviceBatch", train: bool, need_ctx: bool, seed: int):
        if not native.enabled():
            raise NotImplementedError("neighbour attention runs on the native layer executor (U2GNN_NATIVE_LAYER=1)")
        dev = b.X_concat.device
        d, dp = self.d, rup(self.d, 64)
        if not b.input_x.is_contiguous():
            raise ValueError("input_x must be contiguous [N, k+1]")
        W = b.input_x.shape[1]
        dims, tdims = Dims(b.N, d, self.ff), Dims(b.N * W, d, self.ff)
        Np, R, Rp = dims.Np, b.N * W, tdims.Np
        self._pack(dev)
        slot0 = torch.arange(b.N, device=dev, dtype=torch.int64) * W
        X = torch.empty(Rp, dp, device=dev, dtype=torch.float32)
        K.gather_rows(b.X_concat, b.input_x, 1, X, R, Rp, d, dp, b.err)
        outs, lctxs = [], []
        for l in range(self.L):
            lctx = []
            for t in range(self.T):
                seeds = {s: site_seed(seed, l, t, s) for s in (SITE_ATTN, SITE_DROP1, SITE_DROPFF, SITE_DROP2)}
                X, c = native.layer_forward(X, self.packed[l][t], self.layer_params(l, t), tdims, train, seeds,
                                            need_ctx, self.prec, self.p_enc, deep_wgrad=engine_deep_wgrad(), window=W)
                lctx.append(c)
            out = torch.empty(Np, dp, device=dev, dtype=torch.float32)
            K.gather_rows(X, slot0, 1, out, b.N, Np, d, dp)
            outs.append(out)
            lctxs.append(lctx)
            if l + 1 < self.L:
                X = torch.empty(Rp, dp, device=dev, dtype=torch.float32)
                K.gather_rows(out, b.input_x, 1, X, R, Rp, d, dp, b.err)
        return outs, {"dims": dims, "tdims": tdims, "window": W, "slot0": slot0, "layers": lctxs, "batch": b}

    def _backward_neighbors(self, ctx, ext_grad, grads: dict, prefix: str):
        b = ctx["batch"]
        tdims, W, slot0 = ctx["tdims"], ctx["window"], ctx["slot0"]
        d, dp = self.d, rup(self.d, 64)
        R = b.N * W
        off = OffPath(b.input_x.device, enabled=side_stream_pays(tdims))
        dnext = None
        for l in reversed(range(self.L)):
            dOut = ext_grad(l)                                   # [Np, dp] node rows
            if dnext is not None:                                # re-gather of the next U2GNN layer
                K.scatter_add_rows(dnext, b.input_x, 1, dOut, R, d, b.err)
            dX = torch.zeros(tdims.Np, dp, device=dOut.device, dtype=torch.float32)
            K.scatter_add_rows(dOut, slot0, 1, dX, b.N, d)       # slot 0 of every node
            for t in reversed(range(self.T)):
                pre = f"{prefix}.{l}.layers.{t}."
                g = LayerParams(*[grads[pre + k] for k in LAYER_KEYS])
                dX = native.layer_backward(dX, ctx["layers"][l][t], self.packed[l][t], self.layer_params(l, t), g,
                                           tdims, self.prec, side=off.side, deep_wgrad=engine_deep_wgrad(),
                                           need_dx=l > 0 or t > 0)
                self._layer_grads_done(pre, off, need_dx=l > 0 or t > 0)
            dnext = dX
        off.join()
        return dnext

    def _layer_grads_done(self, pre: str, off: OffPath, need_dx: bool) -> None:
        """Hand a layer's finished parameter-gradient region to ``grad_ready`` with a stream ordered after
        EVERY write of that region.  A layer with an input gradient writes its parameter gradients on the
        side stream after a fork from this one (encoder_layer.cpp flush after sd.fork(); engine OffPath.run),
        so the side stream covers them.  The last layer of the backward (need_dx false) writes them on THIS
        stream (encoder_layer.cpp: flush on `st`; engine.py: in_proj_grads inline, the rest on the side
        stream), so the side stream first waits for this one -- nothing is queued behind it any more, so no
        overlap is lost.  Without the wait a collective issued on the side stream read the region before
        the main stream had written it (tests/test_grad_order_gpu.py)."""
        if self.grad_ready is None:
            return
        if not need_dx and off.side is not None:
            off.side.wait_stream(torch.cuda.current_stream())
        self.grad_ready(pre, off.side)

    def backward(self, ctx, ext_grad, grads: dict, prefix: str = "u2gnn_layers"):
        """ext_grad(l) -> fresh padded gradient of outs[l] from outside the stack (head / loss).
        Writes encoder parameter gradients into grads[<reference key>]; returns None (the stack
        input, rows of X_concat, takes no gradient)."""
        if "window" in ctx:
            return self._backward_neighbors(ctx, ext_grad, grads, prefix)
        b = ctx["batch"]
        dims = ctx["dims"]
        dnext = None
        off = OffPath(b.input_x.device, enabled=side_stream_pays(dims))
        for l in reversed(range(self.L)):
            dX = ext_grad(l)
            if dnext is not None:
                K.scatter_add_rows(dnext, b.input_x, b.idx_stride, dX, b.N, self.d, b.err)
            for t in reversed(range(self.T)):
                pre = f"{prefix}.{l}.layers.{t}."
                g = LayerParams(*[grads[pre + k] for k in LAYER_KEYS])
                lc = ctx["layers"][l][t]
                # the stack's input (gathered X_concat rows) is not trainable: no dX out of layer (0, 0)
                need_dx = l > 0 or t > 0
                if isinstance(lc, native.NativeCtx):
                    dX = native.layer_backward(dX, lc, self.packed[l][t], self.layer_params(l, t), g, dims,
                                               self.prec, side=off.side, deep_wgrad=engine_deep_wgrad(),
                                               need_dx=need_dx)
                else:
                    dX = encoder_layer_backward(dX, lc, self.packed[l][t], self.layer_params(l, t), g, dims,
                                                self.prec, off=off, need_dx=need_dx)
                self._layer_grads_done(pre, off, need_dx)
            dnext = dX
        off.join()   # parameter gradients complete before the caller's optimizer reads them
        return dnext


class SupCore:
    """Forward/backward of the supervised TransformerU2GNN (pytorch_U2GNN_Sup.py:30-46)."""

    def __init__(self, module, precision: str = "fp32"):
        self.m = module
        self.prec = precision
        self.d = module.feature_dim_size
        self.ff = module.ff_hidden_size
        self.C = module.num_classes
        self.L = module.num_U2GNN_layers
        self.T = module.num_self_att_layers
        self.p_head = module.dropout_p        # args.dropout, pytorch_U2GNN_Sup.py:28
        # encoder dropout is hard-coded to 0.5 (pytorch_U2GNN_Sup.py:20)
        self.stack = EncoderStack(module.u2gnn_layers, self.d, self.ff, self.T, self.L, precision, 0.5,
                                  getattr(module, "attention", "nodes"))

    def forward(self, b: DeviceBatch, train: bool, need_ctx: bool, seed: int):
        dev = b.X_concat.device
        d, dp = self.d, rup(self.d, 64)
        outs, sctx = self.stack.forward(b, train, need_ctx, seed)
        scores = torch.empty(b.B, self.C, device=dev, dtype=torch.float32)
        ph = self.p_head if train else 0.0
        heads = []
        for l in range(self.L):
            G = torch.empty(b.B, dp, device=dev, dtype=torch.float32)
            hs = site_seed(seed, l, 0, SITE_HEAD)
            K.pool_fwd(outs[l], dp, b.rowptr, b.colidx, b.vals, G, dp, b.B, d, ph, hs)
            K.head_fwd(G, dp, self.m.predictions[l].weight, self.m.predictions[l].bias, scores, b.B, self.C, d,
                       accumulate=l > 0)
            heads.append((G, hs))
        return scores, {"stack": sctx, "heads": heads, "ph": ph, "batch": b}

    def backward(self, ctx, dscores: torch.Tensor, grads: dict):
        """grads: name -> real-shaped tensor (reference state_dict key names)."""
        b: DeviceBatch = ctx["batch"]
        dims: Dims = ctx["stack"]["dims"]
        dev = dscores.device
        d, dp, Np = self.d, dims.dp, dims.Np

        def ext(l):
            G, hs = ctx["heads"][l]
            dG = torch.empty(b.B, dp, device=dev, dtype=torch.float32)
            K.head_bwd(dscores, G, dp, self.m.predictions[l].weight, dG, dp, grads[f"predictions.{l}.weight"],
                       grads[f"predictions.{l}.bias"], b.B, self.C, d)
            if b.block_rows:   # every row stored: no zero fill, no atomics
                dX = torch.empty(Np, dp, device=dev, dtype=torch.float32)
                K.pool_bwd_rows(dG, dp, b.rowptr, b.colidx, b.vals, dX, dp, b.B, d, dp, b.N, Np, ctx["ph"], hs)
            else:
                dX = torch.zeros(Np, dp, device=dev, dtype=torch.float32)
                K.pool_bwd(dG, dp, b.rowptr, b.colidx, b.vals, dX, dp, b.B, d, ctx["ph"], hs)
            return dX
        return self.stack.backward(ctx["stack"], ext, grads)


LAYER_KEYS = ["self_attn.in_proj_weight", "self_attn.in_proj_bias", "self_attn.out_proj.weight",
              "self_attn.out_proj.bias", "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias",
              "norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias"]


class FlatParams:
    """Re-homes every parameter of ``module`` into one flat fp32 device buffer (params become
    views, keeping their reference shapes and state_dict keys) with a matching flat grad buffer."""

    def __init__(self, module: torch.nn.Module, names=None):
        sel = None if names is None else set(names)
        self.names, self.params = zip(*[(n, p) for n, p in module.named_parameters() if sel is None or n in sel])
        dev = self.params[0].device
        sizes = [p.numel() for p in self.params]
        # 16-byte aligned offsets for the float4 sweeps
        offs, o = [], 0
        for s in sizes:
            offs.append(o)
            o += rup(s, 4)
        self.n = o
        self.flat = torch.zeros(o, device=dev, dtype=torch.float32)
        self.gflat = torch.zeros(o, device=dev, dtype=torch.float32)
        self.grads = {}
        for name, p, off, s in zip(self.names, self.params, offs, sizes):
            self.flat[off:off + s].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + s].view(p.shape)
            gv = self.gflat[off:off + s].view(p.shape)
            p.grad = gv
            self.grads[name] = gv


class FusedAdam:
    """torch.optim.Adam (lr, betas=(0.9, 0.999), eps=1e-8, no weight decay) preceded by
    clip_grad_norm_(max_norm) — both on device over the flat buffers, no host sync."""

    def __init__(self, flat: FlatParams, lr: float, max_norm: Optional[float] = 0.5, betas=(0.9, 0.999),
                 eps: float = 1e-8):
        self.f = flat
        self.lr, self.max_norm, self.betas, self.eps = lr, max_norm, betas, eps
        dev = flat.flat.device
        self.m = torch.zeros_like(flat.flat)
        self.v = torch.zeros_like(flat.flat)
        self.ws = torch.empty(1024, device=dev, dtype=torch.float32)
        self.sq = torch.zeros(1, device=dev, dtype=torch.float32)
        self.step_count = 0
        # device-resident schedule (HIP-graph replay, train.StepGraphs): step count t and lr live in
        # HBM, u2gnn_step_advance bumps t inside the captured step, u2gnn_adam_dev forms the bias
        # corrections on the device
        self.t_dev: Optional[torch.Tensor] = None
        self.lr_dev: Optional[torch.Tensor] = None

    def use_device_schedule(self) -> None:
        dev = self.f.flat.device
        self.t_dev = torch.full((1,), self.step_count, device=dev, dtype=torch.int64)
        self.lr_dev = torch.full((1,), float(self.lr), device=dev, dtype=torch.float64)

    def use_host_schedule(self) -> None:
        if self.t_dev is not None:
            self.step_count = int(self.t_dev.item())
        self.t_dev = self.lr_dev = None

    def set_lr(self, lr: float) -> None:
        self.lr = lr
        if self.lr_dev is not None:
            self.lr_dev.fill_(float(lr))

    def step(self):
        b1, b2 = self.betas
        clip = self.max_norm is not None
        if clip:   # the partial sums of g^2; Adam's blocks fold them (u2gnn_adam(_dev)_sq): 2 launches, not 3
            K.sqnorm_partials(self.f.gflat, self.f.n, self.ws)
        if self.t_dev is not None:
            # inside a captured step the graph's first node (StepGraphs: u2gnn_step_advance) bumps t;
            # an eager step taken while the device schedule is live bumps it here, so every path
            # advances t exactly once per step (a fresh t of 0 gave lr / (1 - b1^0) = inf)
            if not torch.cuda.is_current_stream_capturing():
                K.step_advance(None, self.t_dev)
            if clip:
                K.adam_dev_sq(self.f.flat, self.f.gflat, self.m, self.v, self.f.n, self.ws, self.sq, self.max_norm,
                              b1, b2, self.eps, self.lr_dev, self.t_dev)
            else:
                K.adam_dev(self.f.flat, self.f.gflat, self.m, self.v, self.f.n, None, 0.0, b1, b2, self.eps,
                           self.lr_dev, self.t_dev)
            return
        self.step_count += 1
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        if clip:
            K.adam_sq(self.f.flat, self.f.gflat, self.m, self.v, self.f.n, self.ws, self.sq, self.max_norm, b1, b2,
                      self.eps, self.lr / bc1, math.sqrt(bc2))
        else:
            K.adam(self.f.flat, self.f.gflat, self.m, self.v, self.f.n, None, 0.0, b1, b2, self.eps, self.lr / bc1,
                   math.sqrt(bc2))

    def grad_norm(self) -> float:
        return float(self.sq.sqrt().item())
