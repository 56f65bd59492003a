"""Thin torch-tensor wrappers over the C ABI of libu2gnn_hip.so.

Tensors are only used for device memory and stream plumbing: every wrapper passes raw
device pointers + sizes and the current HIP stream to the native entry point, and checks
its status code.  Nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check, hip_lib

PREC = {"fp32": _lib.PREC_F32, "bf16x3": _lib.PREC_BF16X3, "bf16": _lib.PREC_BF16, "bf16x6": _lib.PREC_BF16X6,
        "f16x3": _lib.PREC_F16X3}


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.U2GNNNativeError("U2GNN kernels need device tensors (no CPU fallback)")


class LaunchRecorder:
    """HIP-event bracketing of GEMM launches, keyed by the kernel symbol the launch runs, with the
    launch's ALGORITHMIC FLOPs (real, unpadded dims) supplied by the caller (bench roofline)."""

    def __init__(self):
        self.enabled = False
        self.records = []   # (symbol, flops, start_event, end_event)

    def summary(self):
        """{symbol: (launches, algorithmic flops, milliseconds)} after a synchronize."""
        out = {}
        for sym, fl, s, e in self.records:
            n, f, ms = out.get(sym, (0, 0.0, 0.0))
            out[sym] = (n + 1, f + fl, ms + s.elapsed_time(e))
        return out


REC = LaunchRecorder()
_EPI_NAMES = ["STORE", "BIAS", "BIAS_DROP_RESID", "BIAS_RELU_DROP", "RELU_DROP_BWD", "ACCUM", "ATTN_DS",
              "ATTN_DS_SIGNED"]


def gemm_symbol(precision, M, N, split_k, tile, trans_a, trans_b, epilogue, clamp_a=False):
    """Mirror of the C dispatcher's kernel choice (gemm.hip u2gnn_gemm) -> template symbol."""
    b = lambda x: "true" if x else "false"  # noqa: E731
    if tile == 0:
        can128 = M % 128 == 0 and N % 128 == 0
        tile = 128 if (can128 and (M // 128) * (N // 128) * max(split_k, 1) >= 480) else 64
    b = lambda x: "true" if x else "false"  # noqa: E731
    if precision == "fp32":
        return f"gemm_f32_kernel<{tile}, {tile}, {b(trans_a)}, {b(trans_b)}, {int(epilogue)}, {b(clamp_a)}>"
    # "256" = 256x128 block (4x2 waves); "129" = 128x128 block with a 16-deep K step
    bm, bn, wm, bk = {256: (256, 128, 4, 32), 129: (128, 128, 2, 16)}.get(tile, (tile, tile, 2, 32))
    if precision == "bf16x6":   # three-plane kernel, 16-deep K step on every tile
        return f"gemm_bf16x6_kernel<{bm}, {bn}, {wm}, 2, {b(trans_a)}, {b(trans_b)}, {int(epilogue)}, {b(clamp_a)}>"
    if precision == "f16x3":   # two fp16 planes, the bf16x3 K steps
        return (f"gemm_f16x3_kernel<{bm}, {bn}, {wm}, 2, {bk}, {b(trans_a)}, {b(trans_b)}, {int(epilogue)}, "
                f"{b(clamp_a)}>")
    return (f"gemm_bf16_kernel<{bm}, {bn}, {wm}, 2, {bk}, {b(trans_a)}, {b(trans_b)}, {int(epilogue)}, "
            f"{b(precision == 'bf16x3')}, {b(clamp_a)}>")   # the C++ template instance as rocprofv3 names it


# f16x3 operand pre-scale exponents of the layer executor (encoder_layer.cpp kH3Exp / h3_prob_exp): activations
# and weights (typical magnitudes 2^-5 .. 2^0) by 2^6; the probability image P (entries ~1/N, at most 1/(1-p)) by
# 2^(15 - ceil(log2(1/(1-p)))), so that its largest entry stays below fp16's 65504 and its typical ones keep 22 bits
H3_EXP = 6


def h3_prob_exp(p_drop):
    e, m = 15, 1.0 / (1.0 - float(p_drop))
    while m > 1.0:
        m *= 0.5
        e -= 1
    return e


def gemm(A, B, C, M, N, K, lda, ldb, ldc, trans_a=False, trans_b=False, epilogue=_lib.EPI_STORE, split_k=1,
         slab_stride=0, bias=None, aux0=None, aux1=None, rowvec=None, ld_aux=0, alpha=1.0, scale_cols=0, p_drop=0.0,
         seed=0, precision="fp32", tile=0, flops=None, keep=None, clamp_a=False, Cx2=None, ldcx2=0, cx2_col0=0,
         n_valid=0, ln=None, rowpart=None, h3_exp=None):
    """C[M,N] (epilogue) sum_k A(m,k) B(k,n).  A/B/C may be views (pointer arithmetic via
    storage offsets is done by torch's data_ptr()).  ``flops``: algorithmic FLOPs of the
    launch for the roofline recorder (None = not recorded).  ``clamp_a``: A elements below +0 are read
    as 0 (the signed probability image of attn_softmax_fwd(P=None) consumed as Pd).
    ``Cx2`` (bfloat16) receives the result in x2 format (include/u2gnn_hip.h; columns >= ``cx2_col0``), C may
    then be None.  ``n_valid``: the STORE_ROWSTAT epilogue's real keys.  ``ln`` =
    (gamma, beta, Y, ldy, mean, rstd, d, rows, eps): the EPI_BIAS_DROP_RESID_LN LayerNorm (N == 64).
    ``rowpart`` [N/64, >= M]: the EPI_STORE_ROWDOT row partials (ABI v8).  A 2-D ``rowvec`` [P, >= M]
    gives ATTN_DS_SIGNED the sum of its P partials per row (in row order of ``rowvec``).  ``h3_exp`` = (ea, eb):
    the f16x3 operand pre-scale exponents (ABI v18; None: H3_EXP for both, the layer executor's default)."""
    rec = REC.enabled and flops is not None
    if rec:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    a = _gemm_args(A, B, C, M, N, K, lda, ldb, ldc, trans_a, trans_b, epilogue, split_k, slab_stride, bias, aux0,
                   aux1, rowvec, ld_aux, alpha, scale_cols, p_drop, seed, precision, tile, keep, clamp_a, Cx2, ldcx2,
                   cx2_col0, n_valid, ln, rowpart, h3_exp)
    check(hip_lib().u2gnn_gemm(ctypes.byref(a), _s()), "u2gnn_gemm")
    if rec:
        ev1.record()
        REC.records.append((gemm_symbol(precision, M, N, split_k, tile, trans_a, trans_b, epilogue, clamp_a),
                            float(flops), ev0, ev1))


def gemm_group(calls):
    """Several gemm() calls (each a dict of gemm's keyword arguments; STORE products) in one launch when
    they share a kernel configuration (u2gnn_gemm_group, ABI v11); bit-identical to the separate calls."""
    arr = (_lib.GemmArgs * len(calls))()
    for i, kw in enumerate(calls):
        kw = dict(kw)
        kw.pop("flops", None)
        arr[i] = _gemm_args(**kw)
    check(hip_lib().u2gnn_gemm_group(arr, len(calls), _s()), "u2gnn_gemm_group")


def _gemm_args(A, B, C, M, N, K, lda, ldb, ldc, trans_a=False, trans_b=False, epilogue=_lib.EPI_STORE, split_k=1,
               slab_stride=0, bias=None, aux0=None, aux1=None, rowvec=None, ld_aux=0, alpha=1.0, scale_cols=0,
               p_drop=0.0, seed=0, precision="fp32", tile=0, keep=None, clamp_a=False, Cx2=None, ldcx2=0,
               cx2_col0=0, n_valid=0, ln=None, rowpart=None, h3_exp=None):
    _dev(A, B, C, Cx2)
    if A.dtype != torch.float32 or B.dtype != torch.float32:
        # pre-split (x2) operands were the removed round-1/2 experiments (gemm.hip rejects them)
        raise _lib.U2GNNNativeError("u2gnn_gemm: A and B must be float32 (pre-split operands are not supported)")
    a = _lib.GemmArgs()
    a.A, a.B = A.data_ptr(), B.data_ptr()
    a.C = C.data_ptr() if C is not None else None
    if Cx2 is not None:
        a.Cx2, a.ldcx2, a.cx2_col0 = Cx2.data_ptr(), int(ldcx2), int(cx2_col0)
    a.n_valid = int(n_valid)
    a.M, a.N, a.K = int(M), int(N), int(K)
    a.lda, a.ldb, a.ldc = int(lda), int(ldb), int(ldc)
    a.trans_a, a.trans_b = int(bool(trans_a)), int(bool(trans_b))
    a.epilogue, a.split_k, a.slab_stride = int(epilogue), int(split_k), int(slab_stride)
    a.bias = bias.data_ptr() if bias is not None else None
    a.aux0 = aux0.data_ptr() if aux0 is not None else None
    a.aux1 = aux1.data_ptr() if aux1 is not None else None
    a.rowvec = rowvec.data_ptr() if rowvec is not None else None
    if rowvec is not None and rowvec.dim() == 2:   # ABI v8: partials of a STORE_ROWDOT epilogue
        a.rowvec_parts, a.ld_rowvec = int(rowvec.shape[0]), int(rowvec.stride(0))
    if rowpart is not None:
        _dev(rowpart)
        a.rowpart, a.ld_rowpart = rowpart.data_ptr(), int(rowpart.stride(0))
        if epilogue == _lib.EPI_STORE_ROWSTAT:   # [M, 2 * groups] float32: ld in (max, sum) pairs
            a.ld_rowpart = int(rowpart.stride(0)) // 2
    a.ld_aux = int(ld_aux)
    a.alpha = float(alpha)
    a.scale_cols = int(scale_cols)
    a.p_drop = float(p_drop)
    a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    a.precision = PREC[precision] if isinstance(precision, str) else int(precision)
    a.tile = int(tile)
    if keep is not None:   # ATTN_DS: dropout keep bits (attn_softmax_fwd) instead of Pd
        _dev(keep)
        a.keep, a.ld_keep = keep.data_ptr(), keep.stride(0)
    a.clamp_a = int(bool(clamp_a))
    if h3_exp is not None:
        a.h3_exp_a, a.h3_exp_b = int(h3_exp[0]), int(h3_exp[1])
    elif a.precision == _lib.PREC_F16X3:
        a.h3_exp_a = a.h3_exp_b = H3_EXP
    if ln is not None:
        gam, bet, Y, ldy, mean, rstd, d_real, rows, eps = ln
        _dev(gam, bet, Y, mean, rstd)
        a.ln_gamma, a.ln_beta, a.ln_y, a.ln_ldy = gam.data_ptr(), bet.data_ptr(), Y.data_ptr(), int(ldy)
        a.ln_mean, a.ln_rstd = mean.data_ptr(), rstd.data_ptr()
        a.ln_d, a.ln_rows, a.ln_eps = int(d_real), int(rows), float(eps)
    return a


def gather_rows(src, idx, idx_stride, dst, n_rows, n_rows_pad, d, d_pad, err=None):
    _dev(src, idx, dst)
    check(hip_lib().u2gnn_gather_rows(_p(src), src.stride(0), src.shape[0], _p(idx), int(idx_stride), _p(dst),
                                      dst.stride(0), int(n_rows), int(n_rows_pad), int(d), int(d_pad), _p(err),
                                      _s()), "u2gnn_gather_rows")


def scatter_add_rows(src, idx, idx_stride, dst, n_rows, d, err=None):
    """dst[idx[i]] += src[i] for i < n_rows; out-of-range indices are skipped and flag err (int32[1])."""
    _dev(src, idx, dst)
    check(hip_lib().u2gnn_scatter_add_rows(_p(src), src.stride(0), _p(idx), int(idx_stride), _p(dst), dst.stride(0),
                                           dst.shape[0], int(n_rows), int(d), _p(err), _s()),
          "u2gnn_scatter_add_rows")


def slab_reduce(src, n_slab, slab_stride, rows_pad, cols_pad, ld_src, rblk, cblk, dst, ld_dst, alpha=1.0,
                accumulate=False):
    """rblk/cblk = (blk_pad, blk_real) block maps from padded to real indices."""
    _dev(src, dst)
    check(hip_lib().u2gnn_slab_reduce(_p(src), int(n_slab), int(slab_stride), int(rows_pad), int(cols_pad),
                                      int(ld_src), int(rblk[0]), int(rblk[1]), int(cblk[0]), int(cblk[1]), _p(dst),
                                      int(ld_dst), float(alpha), int(accumulate), _s()), "u2gnn_slab_reduce")


def pack_padded(src, ld_src, rows_pad, cols_pad, rblk, cblk, dst, ld_dst):
    _dev(src, dst)
    check(hip_lib().u2gnn_pack_padded(_p(src), int(ld_src), int(rows_pad), int(cols_pad), int(rblk[0]),
                                      int(rblk[1]), int(cblk[0]), int(cblk[1]), _p(dst), int(ld_dst), _s()),
          "u2gnn_pack_padded")


def reduce_batch(jobs):
    """u2gnn_reduce_batch (ABI v11): a list of dicts of u2gnn_reduce_job fields (tensors for the pointer
    fields); the partial-sum workspace is allocated here.  Bit-identical to the single-job calls."""
    arr = (_lib.ReduceJob * len(jobs))()
    dev = None
    for i, j in enumerate(jobs):
        for k, v in j.items():
            if isinstance(v, torch.Tensor):
                _dev(v)
                dev = v.device
                v = v.data_ptr()
            setattr(arr[i], k, v)
    lib = hip_lib()
    wsf = lib.u2gnn_reduce_batch_ws_floats(arr, len(jobs))
    if wsf < 0:
        raise _lib.U2GNNNativeError("u2gnn_reduce_batch_ws_floats: invalid job")
    ws = torch.empty(max(4, wsf), device=dev, dtype=torch.float32)
    check(lib.u2gnn_reduce_batch(arr, len(jobs), _p(ws), int(wsf), _s()), "u2gnn_reduce_batch")
    return ws


def colsum(X, rows, cols_pad, ld, cblk, out, ws, accumulate=False):
    _dev(X, out, ws)
    check(hip_lib().u2gnn_colsum(_p(X), int(rows), int(cols_pad), int(ld), int(cblk[0]), int(cblk[1]), _p(out),
                                 int(accumulate), _p(ws), _s()), "u2gnn_colsum")


def attn_softmax_fwd(S, lds, P, Pd, ldp, rows_valid, rows_pad, n_valid, n_pad, p, seed, keep=None):
    """keep: optional int32 [rows_pad, >= n_pad/32] receiving the dropout keep bits.  P=None: Pd receives
    the signed image (P/(1-p) where kept, -P where dropped)."""
    _dev(S, Pd, *([t for t in (P, keep) if t is not None]))
    check(hip_lib().u2gnn_attn_softmax_fwd(_p(S), int(lds), _p(P), _p(Pd), int(ldp), int(rows_valid), int(rows_pad),
                                           int(n_valid), int(n_pad), float(p), int(seed), _p(keep),
                                           int(keep.stride(0)) if keep is not None else 0, _s()),
          "u2gnn_attn_softmax_fwd")


def split_x2(src, ld_src, dst2, ld_dst2, rows, cols):
    """dst2 (bfloat16, x2 format) = split of the fp32 rows x cols block of src."""
    _dev(src, dst2)
    check(hip_lib().u2gnn_split_x2(_p(src), int(ld_src), _p(dst2), int(ld_dst2), int(rows), int(cols), _s()),
          "u2gnn_split_x2")


def window_attn_fwd(QKV, W, dp, O, Psave, p, seed, n_nodes, rows_pad):
    """Per-node attention over windows of W token rows (paper semantics); QKV [rows_pad, >=3dp]."""
    _dev(QKV, O, Psave)
    check(hip_lib().u2gnn_window_attn_fwd(_p(QKV), QKV.stride(0), int(W), int(dp), _p(O), O.stride(0), _p(Psave),
                                          float(p), int(seed), int(n_nodes), int(rows_pad), _s()),
          "u2gnn_window_attn_fwd")


def window_attn_bwd(QKV, W, dp, dO, Psave, p, seed, q_scale, dQKV, n_nodes, rows_pad):
    _dev(QKV, dO, Psave, dQKV)
    check(hip_lib().u2gnn_window_attn_bwd(_p(QKV), QKV.stride(0), int(W), int(dp), _p(dO), dO.stride(0), _p(Psave),
                                          float(p), int(seed), float(q_scale), _p(dQKV), dQKV.stride(0),
                                          int(n_nodes), int(rows_pad), _s()), "u2gnn_window_attn_bwd")


def rowdot(A, lda, B, ldb, out, rows, cols):
    _dev(A, B, out)
    check(hip_lib().u2gnn_rowdot(_p(A), int(lda), _p(B), int(ldb), _p(out), int(rows), int(cols), _s()),
          "u2gnn_rowdot")


def layernorm_fwd(Z, ldz, gamma, beta, Y, ldy, mean, rstd, rows_valid, rows_pad, d, d_pad, eps=1e-5):
    _dev(Z, gamma, beta, Y, mean, rstd)
    check(hip_lib().u2gnn_layernorm_fwd(_p(Z), int(ldz), _p(gamma), _p(beta), _p(Y), int(ldy), _p(mean), _p(rstd),
                                        int(rows_valid), int(rows_pad), int(d), int(d_pad), float(eps), _s()),
          "u2gnn_layernorm_fwd")


CS_ROWS = 16   # rows per partial chunk of the column reductions (encoder_ops.hip)


def colstat_ws_floats(rows, cols):
    """Workspace of the two-pass column reductions (colsum, LN parameter gradients)."""
    return max(1, (rows + CS_ROWS - 1) // CS_ROWS) * 3 * cols


def layernorm_bwd(dY, ldy, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, rows_valid, rows_pad, d,
                  d_pad):
    _dev(dY, Z, mean, rstd, gamma, dZ)
    check(hip_lib().u2gnn_layernorm_bwd(_p(dY), int(ldy), _p(Z), int(ldz), _p(mean), _p(rstd), _p(gamma), _p(dZ),
                                        int(lddz), _p(dZdrop), int(lddrop), float(p), int(seed), int(rows_valid),
                                        int(rows_pad), int(d), int(d_pad), _s()), "u2gnn_layernorm_bwd")


def layernorm_bwd_delta_slabs(dY, ldy, slabs, n_slab, slab_stride, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop,
                              lddrop, p, seed, rows_valid, rows_pad, d, d_pad, X, ldx, bias, delta):
    """layernorm_bwd_delta after dY += the split-K slabs (slab_reduce's order, written back; ABI v11)."""
    _dev(dY, slabs, Z, mean, rstd, gamma, dZ, X, bias, delta)
    check(hip_lib().u2gnn_layernorm_bwd_delta_slabs(_p(dY), int(ldy), _p(slabs), int(n_slab), int(slab_stride), _p(Z),
                                                    int(ldz), _p(mean), _p(rstd), _p(gamma), _p(dZ), int(lddz),
                                                    _p(dZdrop), int(lddrop), float(p), int(seed), int(rows_valid),
                                                    int(rows_pad), int(d), int(d_pad), _p(X), int(ldx), _p(bias),
                                                    _p(delta), _s()), "u2gnn_layernorm_bwd_delta_slabs")


def layernorm_bwd_delta(dY, ldy, Z, ldz, mean, rstd, gamma, dZ, lddz, dZdrop, lddrop, p, seed, rows_valid, rows_pad, d,
                        d_pad, X, ldx, bias, delta):
    """layernorm_bwd of an encoder layer's LayerNorm1 that also writes the attention backward's delta
    (rowsum(dO * O) recovered as sum_c dZdrop * ((Z - X)(1-p) - bias); include/u2gnn_hip.h)."""
    _dev(dY, Z, mean, rstd, gamma, dZ, X, bias, delta)
    check(hip_lib().u2gnn_layernorm_bwd_delta(_p(dY), int(ldy), _p(Z), int(ldz), _p(mean), _p(rstd), _p(gamma),
                                              _p(dZ), int(lddz), _p(dZdrop), int(lddrop), float(p), int(seed),
                                              int(rows_valid), int(rows_pad), int(d), int(d_pad), _p(X), int(ldx),
                                              _p(bias), _p(delta), _s()), "u2gnn_layernorm_bwd_delta")


def layernorm_bwd_params(dY, ldy, Z, ldz, mean, rstd, dZdrop, lddrop, rows_valid, d, d_pad, ws, dgamma, dbeta,
                         dbias=None):
    _dev(dY, Z, mean, rstd, ws, dgamma, dbeta)
    check(hip_lib().u2gnn_layernorm_bwd_params(_p(dY), int(ldy), _p(Z), int(ldz), _p(mean), _p(rstd), _p(dZdrop),
                                               int(lddrop), int(rows_valid), int(d), int(d_pad), _p(ws), _p(dgamma),
                                               _p(dbeta), _p(dbias), _s()), "u2gnn_layernorm_bwd_params")


# a step advance (epoch, t) handed to the next weight pack (train.StepGraphs: the replayed step's first node
# rides on its first launch instead of a launch of its own)
_PENDING_ADVANCE = []


def defer_step_advance(epoch, t):
    _dev(epoch, t)
    _PENDING_ADVANCE[:] = [(epoch, t)]


def step_advance_pending() -> bool:
    return bool(_PENDING_ADVANCE)


def pack_padded_multi(jobs):
    """jobs: list of (src, ld_src, rows_pad, cols_pad, rblk, cblk, dst, ld_dst)."""
    arr = (_lib.PackDesc * len(jobs))()
    for i, (src, ld_src, rp, cp, rb, cb, dst, ld_dst) in enumerate(jobs):
        _dev(src, dst)
        arr[i] = _lib.PackDesc(src.data_ptr(), dst.data_ptr(), int(ld_src), int(rp), int(cp), int(rb[0]), int(rb[1]),
                               int(cb[0]), int(cb[1]), int(ld_dst))
    if _PENDING_ADVANCE and jobs:
        epoch, t = _PENDING_ADVANCE.pop()
        check(hip_lib().u2gnn_pack_padded_multi_adv(arr, len(jobs), _p(epoch), _p(t), _s()),
              "u2gnn_pack_padded_multi_adv")
        return
    check(hip_lib().u2gnn_pack_padded_multi(arr, len(jobs), _s()), "u2gnn_pack_padded_multi")


def pool_fwd(X, ldx, rowptr, colidx, vals, G, ldg, B, d, p, seed):
    _dev(X, rowptr, colidx, vals, G)
    check(hip_lib().u2gnn_pool_fwd(_p(X), int(ldx), _p(rowptr), _p(colidx), _p(vals), _p(G), int(ldg), int(B),
                                   int(d), float(p), int(seed), _s()), "u2gnn_pool_fwd")


def pool_bwd_rows(dG, ldg, rowptr, colidx, vals, dX, ldx, B, d, d_pad, N, rows_pad, p, seed):
    """Block-row pool backward with plain stores (every row of dX[:rows_pad, :d_pad] written)."""
    _dev(dG, rowptr, colidx, vals, dX)
    check(hip_lib().u2gnn_pool_bwd_rows(_p(dG), int(ldg), _p(rowptr), _p(colidx), _p(vals), _p(dX), int(ldx), int(B),
                                        int(d), int(d_pad), int(N), int(rows_pad), float(p), int(seed), _s()),
          "u2gnn_pool_bwd_rows")


def pool_bwd(dG, ldg, rowptr, colidx, vals, dX, ldx, B, d, p, seed):
    _dev(dG, rowptr, colidx, vals, dX)
    check(hip_lib().u2gnn_pool_bwd(_p(dG), int(ldg), _p(rowptr), _p(colidx), _p(vals), _p(dX), int(ldx), int(B),
                                   int(d), float(p), int(seed), _s()), "u2gnn_pool_bwd")


def head_fwd(G, ldg, W, bias, scores, B, C, d, accumulate):
    _dev(G, W, bias, scores)
    check(hip_lib().u2gnn_head_fwd(_p(G), int(ldg), _p(W), _p(bias), _p(scores), int(B), int(C), int(d),
                                   int(accumulate), _s()), "u2gnn_head_fwd")


def head_bwd(dscores, G, ldg, W, dG, lddg, dW, db, B, C, d, accumulate=False):
    _dev(dscores, G, W, dG, dW, db)
    check(hip_lib().u2gnn_head_bwd(_p(dscores), _p(G), int(ldg), _p(W), _p(dG), int(lddg), _p(dW), _p(db), int(B),
                                   int(C), int(d), int(accumulate), _s()), "u2gnn_head_bwd")


def smoothed_ce(scores, labels, B, C, smoothing, loss, dscores):
    _dev(scores, labels, loss, dscores)
    check(hip_lib().u2gnn_smoothed_ce(_p(scores), _p(labels), int(B), int(C), float(smoothing), _p(loss),
                                      _p(dscores), _s()), "u2gnn_smoothed_ce")


def sqnorm_partials(g, n, ws):
    """Per-block partial sums of g^2 into ws (ABI v11; folded by adam_sq / adam_dev_sq)."""
    _dev(g, ws)
    check(hip_lib().u2gnn_sqnorm_partials(_p(g), int(n), _p(ws), _s()), "u2gnn_sqnorm_partials")


def adam_sq(param, grad, m, v, n, ws, sq_out, max_norm, beta1, beta2, eps, step_size, bc2_sqrt):
    """Clip + Adam with the sqnorm partials folded in (ABI v11); sq_out receives sum g^2."""
    _dev(param, grad, m, v, ws, sq_out)
    check(hip_lib().u2gnn_adam_sq(_p(param), _p(grad), _p(m), _p(v), int(n), _p(ws), _p(sq_out), float(max_norm),
                                  float(beta1), float(beta2), float(eps), float(step_size), float(bc2_sqrt), _s()),
          "u2gnn_adam_sq")


def adam_dev_sq(param, grad, m, v, n, ws, sq_out, max_norm, b1, b2, eps, lr_dev, step_dev):
    """adam_dev with the sqnorm partials folded in (ABI v11)."""
    _dev(param, grad, m, v, ws, sq_out, lr_dev, step_dev)
    check(hip_lib().u2gnn_adam_dev_sq(_p(param), _p(grad), _p(m), _p(v), int(n), _p(ws), _p(sq_out), float(max_norm),
                                      float(b1), float(b2), float(eps), _p(lr_dev), _p(step_dev), _s()),
          "u2gnn_adam_dev_sq")


def sqnorm(g, n, ws, out):
    _dev(g, ws, out)
    check(hip_lib().u2gnn_sqnorm(_p(g), int(n), _p(ws), _p(out), _s()), "u2gnn_sqnorm")


def adam(param, grad, m, v, n, sqnorm_t, max_norm, beta1, beta2, eps, step_size, bc2_sqrt):
    _dev(param, grad, m, v)
    check(hip_lib().u2gnn_adam(_p(param), _p(grad), _p(m), _p(v), int(n), _p(sqnorm_t), float(max_norm),
                               float(beta1), float(beta2), float(eps), float(step_size), float(bc2_sqrt), _s()),
          "u2gnn_adam")


def sampled_softmax_fwd(X, ldx, labels, sample_ids, S, W, ldw, loss, prob, n_rows, D):
    _dev(X, labels, sample_ids, W, loss, prob)
    check(hip_lib().u2gnn_sampled_softmax_fwd(_p(X), int(ldx), _p(labels), _p(sample_ids), int(S), _p(W), int(ldw),
                                              _p(loss), _p(prob), int(n_rows), int(D), _s()),
          "u2gnn_sampled_softmax_fwd")


def sampled_softmax_bwd(X, ldx, labels, sample_ids, S, W, ldw, prob, dloss, dX, lddx, dW, lddw, n_rows, D):
    _dev(X, labels, sample_ids, W, prob, dX, dW)
    check(hip_lib().u2gnn_sampled_softmax_bwd(_p(X), int(ldx), _p(labels), _p(sample_ids), int(S), _p(W), int(ldw),
                                              _p(prob), _p(dloss), _p(dX), int(lddx), _p(dW), int(lddw), int(n_rows),
                                              int(D), _s()), "u2gnn_sampled_softmax_bwd")


def attn_softmax_pv_ws_floats(n_valid, rows_pad, dp):
    return int(hip_lib().u2gnn_attn_softmax_pv_ws_floats(int(n_valid), int(rows_pad), int(dp)))


def attn_softmax_pv(S, lds, rowpart, ngroups, qkv2, ldq2, dp, Pd, ldp, O, ldo, ws, n_valid, rows_pad, p, seed,
                    precision="bf16x3"):
    """ABI v10: signed probability image Pd and O = dropout(P) V from the scores S, the EPI_STORE_ROWSTAT
    row partials ``rowpart`` (float32 [rows, >= 2*ngroups]) and the x2 in-projection output qkv2 (bfloat16); with
    precision "bf16x6" (ABI v17) qkv2 is the fp32 in-projection output and ldq2 its row length in floats."""
    _dev(S, rowpart, qkv2, Pd, O, ws)
    check(hip_lib().u2gnn_attn_softmax_pv(_p(S), int(lds), _p(rowpart), int(rowpart.stride(0)) // 2, int(ngroups),
                                          _p(qkv2), int(ldq2), int(dp), _p(Pd), int(ldp), _p(O), int(ldo), _p(ws),
                                          int(ws.numel()), int(n_valid), int(rows_pad), float(p),
                                          int(seed) & 0xFFFFFFFFFFFFFFFF, PREC[precision], _s()),
          "u2gnn_attn_softmax_pv")


def attn_small_ctx_floats(rows_pad, d):
    return int(hip_lib().u2gnn_attn_small_ctx_floats(int(rows_pad), int(d)))


def attn_small_ws_floats(n_valid, rows_pad, d):
    return int(hip_lib().u2gnn_attn_small_ws_floats(int(n_valid), int(rows_pad), int(d)))


def attn_small_fwd(X, ldx, W_in, b_in, dp, d, n_valid, rows_pad, p, seed, O, ldo, ctx):
    """ABI v15 (d <= 32): the in-projection of X (W_in [3 dp, dp], b_in [3 dp] padded) and O = dropout(softmax(Q
    K^T)) V on the vector ALUs, flash-style, with the forward context ctx [attn_small_ctx_floats(rows_pad, d)]:
    the row statistics ctx[:2 rows_pad].view(rows_pad, 2) = (max log2 e, 1 / sum exp) the backward recomputes P
    from, then a compact copy of Q (scaled by 1/sqrt(d)), K, V."""
    _dev(X, W_in, b_in, O, ctx)
    check(hip_lib().u2gnn_attn_small_fwd(_p(X), int(ldx), _p(W_in), _p(b_in), int(dp), int(d), int(n_valid),
                                         int(rows_pad), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, _p(O), int(ldo),
                                         _p(ctx), int(ctx.numel()), _s()), "u2gnn_attn_small_fwd")


def attn_small_bwd(ctx, W_in, dp, d, n_valid, rows_pad, p, seed, dO, ld_do, delta, q_scale, dQKV, ld_dqkv, dX, lddx,
                   ws):
    """ABI v15 (d <= 32): dQKV = (q_scale dS K, dS^T Q, Pd^T dO) with P recomputed from the forward's ctx, and
    dX += dQKV W_in unless dX is None."""
    _dev(ctx, W_in, dO, delta, dQKV, dX, ws)
    check(hip_lib().u2gnn_attn_small_bwd(_p(ctx), int(ctx.numel()), _p(W_in), int(dp), int(d), int(n_valid),
                                         int(rows_pad), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, _p(dO), int(ld_do),
                                         _p(delta), float(q_scale), _p(dQKV), int(ld_dqkv), _p(dX), int(lddx),
                                         _p(ws), int(ws.numel()), _s()), "u2gnn_attn_small_bwd")


def _tail_args(N, Np, d, dp, ff, ffp, p, seeds, t):
    _dev(*t.values())
    a = _lib.SmallTailArgs()
    a.n_valid, a.rows_pad, a.d, a.dp, a.ff, a.ffp = int(N), int(Np), int(d), int(dp), int(ff), int(ffp)
    a.p, a.eps = float(p), 1e-5
    a.seed_drop1, a.seed_dropff, a.seed_drop2 = [int(x) & 0xFFFFFFFFFFFFFFFF for x in seeds]
    for k, v in t.items():
        if k not in _lib._TAIL_PTRS:
            raise _lib.U2GNNNativeError(f"small-width layer: unknown tensor {k}")
        setattr(a, k, None if v is None else v.data_ptr())
    return a


def layer_tail_small(backward, N, Np, d, dp, ff, ffp, p, seeds, **t):
    """ABI v15 (d <= 32): the row-local tail of an encoder layer in one launch each way (small_layer.hip).
    seeds = (drop1, dropff, drop2); t: the tensors of u2gnn_small_tail_args by field name (weights in the
    padded layouts, LayerNorm parameters [d]).  Forward: O, X -> Z1, X1, mean1, rstd1, Hd, Z2, X2, mean2, rstd2;
    backward: dX2 and the forward tensors -> dX1, dF, dH, dX, dA, dO, delta."""
    a = _tail_args(N, Np, d, dp, ff, ffp, p, seeds, t)
    fn = hip_lib().u2gnn_layer_tail_small_bwd if backward else hip_lib().u2gnn_layer_tail_small_fwd
    check(fn(ctypes.byref(a), _s()), "u2gnn_layer_tail_small_" + ("bwd" if backward else "fwd"))


def layer_tail_mid_ws_floats(Np, dp, ffp):
    return int(hip_lib().u2gnn_layer_tail_mid_ws_floats(int(Np), int(dp), int(ffp)))


def layer_tail_mid_fwd(N, Np, d, dp, ff, ffp, p, seeds, ws, **t):
    """ABI v16 (d <= 256): the forward tail of a mid-width layer -- out-projection .. LayerNorm2 -- in two launches
    (mid_layer.hip + the slab LayerNorm); t: the forward tensors of u2gnn_small_tail_args; ws: the chunk slabs."""
    _dev(ws)
    a = _tail_args(N, Np, d, dp, ff, ffp, p, seeds, t)
    check(hip_lib().u2gnn_layer_tail_mid_fwd(ctypes.byref(a), _p(ws), int(ws.numel()), _s()), "u2gnn_layer_tail_mid_fwd")


def layer_small_fwd(N, Np, d, dp, ff, ffp, p, seeds, attn_seed, W_in, b_in, ctx, **t):
    """ABI v15 (d <= 32): the whole layer forward -- in-projection, node attention (O into t["O"], the attention
    context into ctx) and the tail -- in 2 or 3 launches (attention and tail fused from 1024 padded rows)."""
    _dev(W_in, b_in, ctx)
    a = _tail_args(N, Np, d, dp, ff, ffp, p, seeds, t)
    check(hip_lib().u2gnn_layer_small_fwd(ctypes.byref(a), _p(W_in), _p(b_in), int(attn_seed) & 0xFFFFFFFFFFFFFFFF,
                                          _p(ctx), int(ctx.numel()), _s()), "u2gnn_layer_small_fwd")


def layer_small_bwd(N, Np, d, dp, ff, ffp, p, seeds, attn_seed, W_in, ctx, dQKV, accumulate_dx, ws, **t):
    """ABI v15 (d <= 32): the whole layer backward -- the tail backward (t: dX1, dF, dH, dX, dA, dO, delta) and the
    attention backward (dQKV [rows_pad, 3 dp]; t["dX"] += dQKV W_in when accumulate_dx) in 2 or 3 launches."""
    _dev(W_in, ctx, dQKV, ws)
    a = _tail_args(N, Np, d, dp, ff, ffp, p, seeds, t)
    check(hip_lib().u2gnn_layer_small_bwd(ctypes.byref(a), _p(W_in), int(attn_seed) & 0xFFFFFFFFFFFFFFFF, _p(ctx),
                                          int(ctx.numel()), _p(dQKV), int(dQKV.stride(0)), 1 if accumulate_dx else 0,
                                          _p(ws), int(ws.numel()), _s()), "u2gnn_layer_small_bwd")


def sampled_softmax_bwd_rows(X, ldx, labels, sample_ids, S, W, ldw, prob, dloss, dX, lddx, dW_lab, dW_smp, n_rows, D):
    """ABI v9: W's gradient as compact rows -- dW_lab [n_rows, >= D] (row of W labels[i]) and dW_smp
    [S, >= D] (row of W sample_ids[j]) -- instead of a dense [V, D] image."""
    _dev(X, labels, sample_ids, W, prob, dX, dW_smp, dW_lab)
    check(hip_lib().u2gnn_sampled_softmax_bwd_rows(_p(X), int(ldx), _p(labels), _p(sample_ids), int(S), _p(W), int(ldw),
                                                   _p(prob), _p(dloss), _p(dX), int(lddx), _p(dW_lab),
                                                   int(dW_lab.stride(0)) if dW_lab is not None else int(D), _p(dW_smp),
                                                   int(dW_smp.stride(0)), int(n_rows), int(D), _s()),
          "u2gnn_sampled_softmax_bwd_rows")


def index_add_rows(src, idx, dst, alpha=1.0, err=None):
    """dst[idx[r]] += alpha * src[r] (idx distinct within one call; u2gnn_hip.h ABI v9)."""
    _dev(src, idx, dst, err)
    n, D = int(idx.numel()), int(dst.shape[1])
    check(hip_lib().u2gnn_index_add_rows(_p(src), int(src.stride(0)), _p(idx), n, float(alpha), _p(dst),
                                         int(dst.stride(0)), int(dst.shape[0]), D, _p(err), _s()),
          "u2gnn_index_add_rows")


def index_zero_rows(idx, dst, err=None):
    """dst[idx[r]] = 0 (ABI v9)."""
    _dev(idx, dst, err)
    check(hip_lib().u2gnn_index_zero_rows(_p(idx), int(idx.numel()), _p(dst), int(dst.stride(0)), int(dst.shape[0]),
                                          int(dst.shape[1]), _p(err), _s()), "u2gnn_index_zero_rows")


def index_zero_rows2(idx_a, idx_b, dst, err=None):
    """dst[idx_a[r]] = 0 and dst[idx_b[r]] = 0 in one launch (ABI v11)."""
    _dev(idx_a, idx_b, dst, err)
    check(hip_lib().u2gnn_index_zero_rows2(_p(idx_a), int(idx_a.numel()), _p(idx_b), int(idx_b.numel()), _p(dst),
                                           int(dst.stride(0)), int(dst.shape[0]), int(dst.shape[1]), _p(err), _s()),
          "u2gnn_index_zero_rows2")


def concat_dropout(srcs, ld_src, N, d, Y, ldy, p, seed):
    """Y[:, l*d:(l+1)*d] = drop(srcs[l][:N, :d]) over Y's indices (ABI v11)."""
    _dev(*srcs, Y)
    arr = (ctypes.c_void_p * len(srcs))(*[t.data_ptr() for t in srcs])
    check(hip_lib().u2gnn_concat_dropout(arr, len(srcs), int(ld_src), int(N), int(d), float(p), int(seed), _p(Y),
                                         int(ldy), _s()), "u2gnn_concat_dropout")


def split_dropout_bwd(dY, ldy, N, Np, d, dp, p, seed, dsts):
    """dsts[l] ([Np, dp], contiguous) = zero-padded drop(dY[:, l*d:(l+1)*d]) (ABI v11)."""
    _dev(dY, *dsts)
    arr = (ctypes.c_void_p * len(dsts))(*[t.data_ptr() for t in dsts])
    check(hip_lib().u2gnn_split_dropout_bwd(_p(dY), int(ldy), len(dsts), int(N), int(Np), int(d), int(dp), float(p),
                                            int(seed), arr, _s()), "u2gnn_split_dropout_bwd")


def slab_bias_drop_resid_ln(slabs, n_slab, slab_stride, bias, resid, p, seed, Z, gamma, beta, Y, mean, rstd, d,
                            rows_valid, rows_pad, eps=1e-5):
    """FFN2's split-K epilogue (ABI v11; d <= 256 since round 5): Z = resid + drop(sum of slabs + bias), Y = LN(Z).
    slabs [n_slab, rows_pad, dp]; resid, Z, Y [rows_pad, dp] with dp = rup(d, 64)."""
    _dev(slabs, bias, resid, Z, gamma, beta, Y, mean, rstd)
    dp = -(-int(d) // 64) * 64
    check(hip_lib().u2gnn_slab_bias_drop_resid_ln(_p(slabs), int(n_slab), int(slab_stride), dp, _p(bias), _p(resid),
                                                  int(resid.stride(0)), float(p), int(seed), _p(Z), int(Z.stride(0)),
                                                  _p(gamma), _p(beta), _p(Y), int(Y.stride(0)), _p(mean), _p(rstd),
                                                  int(d), int(rows_valid), int(rows_pad), float(eps), _s()),
          "u2gnn_slab_bias_drop_resid_ln")


def sum_all(x, n, out):
    """out[0] = sum of the first n elements of x, fixed order, one launch (ABI v11)."""
    _dev(x, out)
    check(hip_lib().u2gnn_sum(_p(x), int(n), _p(out), _s()), "u2gnn_sum")


def dropout(X, ldx, Y, ldy, rows, cols, p, seed):
    _dev(X, Y)
    check(hip_lib().u2gnn_dropout(_p(X), int(ldx), _p(Y), int(ldy), int(rows), int(cols), float(p), int(seed), _s()),
          "u2gnn_dropout")


def dropout_mask(seed, rows, cols, p, device="cuda"):
    out = torch.empty(rows, cols, dtype=torch.uint8, device=device)
    check(hip_lib().u2gnn_dropout_mask(int(seed), int(rows), int(cols), float(p), _p(out), _s()),
          "u2gnn_dropout_mask")
    return out


# ---- ABI v6: device-resident step state for HIP-graph replay (u2gnn_hip.h) ----
def set_seed_epoch(epoch):
    """Every dropout-drawing launch from now on mixes the device uint64 ``epoch[0]`` into its seed
    (None switches it off).  Process-wide."""
    if epoch is not None:
        _dev(epoch)
        if epoch.dtype != torch.int64 or epoch.numel() < 1:
            raise _lib.U2GNNNativeError("seed epoch: one int64 device element")
    check(hip_lib().u2gnn_set_seed_epoch(_p(epoch) if epoch is not None else None), "u2gnn_set_seed_epoch")


def step_advance(epoch, step):
    """epoch[0] += 1 and step[0] += 1 on the current stream (either may be None)."""
    check(hip_lib().u2gnn_step_advance(_p(epoch) if epoch is not None else None,
                                       _p(step) if step is not None else None, _s()), "u2gnn_step_advance")


def adam_dev(param, grad, m, v, n, sqnorm, max_norm, b1, b2, eps, lr_dev, step_dev):
    """u2gnn_adam with the bias corrections formed on the device from lr_dev (float64[1]) and
    step_dev (int64[1])."""
    _dev(param, grad, m, v, lr_dev, step_dev)
    check(hip_lib().u2gnn_adam_dev(_p(param), _p(grad), _p(m), _p(v), int(n), _p(sqnorm) if sqnorm is not None else None,
                                   float(max_norm), float(b1), float(b2), float(eps), _p(lr_dev), _p(step_dev), _s()),
          "u2gnn_adam_dev")
