"""Python handle on the native encoder-layer executor (csrc/encoder_layer.cpp,
include/u2gnn_hip.h u2gnn_layer_*): one C-ABI call per layer forward / backward.

engine.py issues the same kernel sequence launch by launch from Python (kept as the readable
reference orchestration and for per-GEMM event timing); this module is the production path.
Buffers come from the torch caching allocator: the forward's saved tensors live in one uint8
"ctx" tensor per layer, workspaces are allocated per call.  Memory read by the backward's
side stream is record_stream'ed so the allocator cannot recycle it early.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch

from . import _lib
from ._lib import LayerDims, LayerGrads, LayerParamsC, LayerSeeds, check, hip_lib
from .kernels import PREC

_SIZES: Dict[tuple, tuple] = {}


_ENABLED = [os.environ.get("U2GNN_NATIVE_LAYER", "1") == "1"]


def enabled() -> bool:
    """U2GNN_NATIVE_LAYER=0 routes layers through the Python orchestration (engine.py)."""
    return _ENABLED[0]


def set_enabled(on: bool) -> bool:
    """bench.py's per-GEMM timing pass runs the Python orchestration (its wrappers carry the HIP
    events); returns the previous setting."""
    prev = _ENABLED[0]
    _ENABLED[0] = bool(on)
    return prev


def _dims(N: int, d: int, ff: int, prec: str, deep_wgrad: bool, window: int = 0) -> LayerDims:
    flags = _lib.LAYER_DEEP_WGRAD if deep_wgrad else 0
    if prec == "mixed":   # bf16x3 except the attention-backward products dS, dQ, dK (engine.MIXED_BF16_ROLES)
        prec, flags = "bf16x3", flags | _lib.LAYER_ATTN_BWD_BF16
    elif prec == "fwd32":  # exact fp32 forward products, bf16x3 backward (engine.FWD_ROLES)
        prec, flags = "bf16x3", flags | _lib.LAYER_FWD_F32
    elif prec == "fwd6":   # bf16x6 forward products, bf16x3 backward (engine.FWD_ROLES)
        prec, flags = "bf16x3", flags | _lib.LAYER_FWD_X6
    elif prec == "fwdh":   # f16x3 forward products, bf16x3 backward (engine.FWD_ROLES)
        prec, flags = "bf16x3", flags | _lib.LAYER_FWD_H3
    return LayerDims(int(N), int(d), int(ff), PREC[prec], flags, int(window), 0)


def sizes(N: int, d: int, ff: int, prec: str, p_drop: float, deep_wgrad: bool = True, window: int = 0):
    key = (N, d, ff, prec, p_drop > 0, deep_wgrad, window)
    r = _SIZES.get(key)
    if r is None:
        c, f, b = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        dims = _dims(N, d, ff, prec, deep_wgrad, window)
        check(hip_lib().u2gnn_layer_sizes(ctypes.byref(dims), float(p_drop), ctypes.byref(c), ctypes.byref(f),
                                          ctypes.byref(b)), "u2gnn_layer_sizes")
        r = _SIZES[key] = (c.value, f.value, b.value)
    return r


def _params(packed, p) -> LayerParamsC:
    return LayerParamsC(packed.W_in.data_ptr(), packed.b_in.data_ptr(), packed.W_o.data_ptr(), packed.b_o.data_ptr(),
                        packed.W1.data_ptr(), packed.b1.data_ptr(), packed.W2.data_ptr(), packed.b2.data_ptr(),
                        p.n1_w.data_ptr(), p.n1_b.data_ptr(), p.n2_w.data_ptr(), p.n2_b.data_ptr())


def _seeds(p_drop: float, seeds: Dict[int, int]) -> LayerSeeds:
    from .engine import SITE_ATTN, SITE_DROP1, SITE_DROP2, SITE_DROPFF
    return LayerSeeds(float(p_drop), seeds.get(SITE_ATTN, 0), seeds.get(SITE_DROP1, 0), seeds.get(SITE_DROPFF, 0),
                      seeds.get(SITE_DROP2, 0))


class NativeCtx:
    """What the backward needs from one layer's forward."""
    __slots__ = ("X", "buf", "p_drop", "seeds", "window")


def _stream(s=None):
    return ctypes.c_void_p((s or torch.cuda.current_stream()).cuda_stream)


def layer_forward(X: torch.Tensor, packed, p, dims, train: bool, seeds: Dict[int, int], need_ctx: bool,
                  prec: str, p_enc: float, deep_wgrad: bool = True, window: int = 0):
    """window = 0: attention over all dims.N rows; W: within each node's window of W token rows
    (dims.N = nodes * W)."""
    pd = p_enc if train else 0.0
    cb, fb, _ = sizes(dims.N, dims.d, dims.ff, prec, pd, deep_wgrad, window)
    dev = X.device
    X2 = torch.empty(dims.Np, dims.dp, device=dev, dtype=torch.float32)
    buf = torch.empty(cb, device=dev, dtype=torch.uint8) if need_ctx else None
    ws = torch.empty(max(256, fb + (0 if need_ctx else cb)), device=dev, dtype=torch.uint8)
    dd, pp, ss = _dims(dims.N, dims.d, dims.ff, prec, deep_wgrad, window), _params(packed, p), _seeds(pd, seeds)
    check(hip_lib().u2gnn_layer_fwd(ctypes.byref(dd), ctypes.byref(pp), ctypes.byref(ss), X.data_ptr(),
                                    X2.data_ptr(), buf.data_ptr() if buf is not None else None, cb,
                                    ws.data_ptr(), ws.numel(), _stream()), "u2gnn_layer_fwd")
    ctx = None
    if need_ctx:
        ctx = NativeCtx()
        ctx.X, ctx.buf, ctx.p_drop, ctx.seeds, ctx.window = X, buf, pd, dict(seeds), window
    return X2, ctx


def layer_backward(dX2: torch.Tensor, ctx: NativeCtx, packed, p, g, dims, prec: str,
                   side: Optional["torch.cuda.Stream"] = None, deep_wgrad: bool = True,
                   need_dx: bool = True) -> Optional[torch.Tensor]:
    cb, _, bb = sizes(dims.N, dims.d, dims.ff, prec, ctx.p_drop, deep_wgrad, ctx.window)
    dev = dX2.device
    dX = torch.empty(dims.Np, dims.dp, device=dev, dtype=torch.float32) if need_dx else None
    ws = torch.empty(max(256, bb), device=dev, dtype=torch.uint8)
    dd = _dims(dims.N, dims.d, dims.ff, prec, deep_wgrad, ctx.window)
    pp, ss = _params(packed, p), _seeds(ctx.p_drop, ctx.seeds)
    gg = LayerGrads(*[getattr(g, k).data_ptr() for k in _lib._PKEYS])
    check(hip_lib().u2gnn_layer_bwd(ctypes.byref(dd), ctypes.byref(pp), ctypes.byref(ss), ctx.X.data_ptr(),
                                    ctx.buf.data_ptr(), cb, dX2.data_ptr(), dX.data_ptr() if need_dx else None, ctypes.byref(gg),
                                    ws.data_ptr(), ws.numel(), _stream(), _stream(side) if side is not None else None),
          "u2gnn_layer_bwd")
    if side is not None:
        for t in (ws, ctx.buf, ctx.X, dX2):
            t.record_stream(side)
    return dX


def probe_arm(role: int, capacity: int) -> None:
    """Time the next `capacity` executor launches of one product (``_lib.ROLE_*``) with HIP events
    recorded on the stream each kernel runs on (u2gnn_probe_arm)."""
    check(hip_lib().u2gnn_probe_arm(int(role), int(capacity)), "u2gnn_probe_arm")


def probe_collect():
    """(summed device milliseconds, launches) of the armed probe; frees its events."""
    ms, n = ctypes.c_float(), ctypes.c_int32()
    check(hip_lib().u2gnn_probe_collect(ctypes.byref(ms), ctypes.byref(n)), "u2gnn_probe_collect")
    return float(ms.value), int(n.value)
