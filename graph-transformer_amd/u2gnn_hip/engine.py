"""U2GNN forward / backward engine on the gfx950 kernels.

Reference semantics: the reference feeds ``F.embedding(input_x, X_concat)``
[N, k+1, d] to ``nn.TransformerEncoder`` with ``batch_first=False``
(pytorch_U2GNN_Sup.py:32,35), so the attention sequence is the N nodes of the batch and the
k+1 neighbour slots are independent batch entries of which only slot 0 is kept
(:36-37).  Slot 0 is row i itself (``input_x[:,0] == arange(N)``).  This engine therefore
computes exactly the slot-0 path — gather(X_concat, input_x[:,0]) -> T post-LN encoder
layers with single-head attention over all N nodes -> pooling/head — which is equal to the
reference output (slots 1..k never reach the output) at 1/(k+1) of the reference's work.

Layouts in HBM (fp32, row-major): node rows padded to Np = row_pad(N) (a multiple of 128, of 256
from 1024 rows on), feature columns
to dp = roundup(d, 64), FFN width to ffp = roundup(ff, 64); QKV is one [Np, 3*dp] buffer
(Q pre-scaled by 1/sqrt(d)); the attention probabilities are one [Np, Np] image (with dropout the
signed one: P/(1-p) where kept, -P where dropped).
Padding rows/columns hold zeros in every activation and gradient the encoder produces
(invariant relied upon by the GEMMs, which run on the padded shapes without masks).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from . import _lib
from . import kernels as K

E = _lib


def rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def row_pad(N: int) -> int:
    """Padded node rows: multiples of 256 from 1024 rows on (the N^2 products then always run on
    256x128 blocks), else of 128.  Mirrors rows_pad() in csrc/encoder_layer.cpp."""
    return rup(N, 256) if N >= 1024 else rup(N, 128)


def _mix64(z: int) -> int:
    z &= 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def site_seed(base: int, *ids: int) -> int:
    s = base & 0xFFFFFFFFFFFFFFFF
    for i in ids:
        s = _mix64(s + 0x9E3779B97F4A7C15 * (i + 1))
    return s


# dropout sites inside one encoder layer
SITE_ATTN, SITE_DROP1, SITE_DROPFF, SITE_DROP2 = 1, 2, 3, 4
SITE_HEAD = 5


@dataclass
class Dims:
    N: int
    d: int
    ff: int

    @property
    def Np(self):
        return row_pad(self.N)

    @property
    def dp(self):
        return rup(self.d, 64)

    @property
    def ffp(self):
        return rup(self.ff, 64)


@dataclass
class LayerParams:
    """Real-shaped parameter tensors of one torch TransformerEncoderLayer (reference keys)."""
    in_w: torch.Tensor
    in_b: torch.Tensor
    out_w: torch.Tensor
    out_b: torch.Tensor
    l1_w: torch.Tensor
    l1_b: torch.Tensor
    l2_w: torch.Tensor
    l2_b: torch.Tensor
    n1_w: torch.Tensor
    n1_b: torch.Tensor
    n2_w: torch.Tensor
    n2_b: torch.Tensor

    @staticmethod
    def from_encoder_layer(layer) -> "LayerParams":
        return LayerParams(layer.self_attn.in_proj_weight, layer.self_attn.in_proj_bias,
                           layer.self_attn.out_proj.weight, layer.self_attn.out_proj.bias,
                           layer.linear1.weight, layer.linear1.bias, layer.linear2.weight, layer.linear2.bias,
                           layer.norm1.weight, layer.norm1.bias, layer.norm2.weight, layer.norm2.bias)

    def tensors(self) -> List[torch.Tensor]:
        return [self.in_w, self.in_b, self.out_w, self.out_b, self.l1_w, self.l1_b, self.l2_w, self.l2_b,
                self.n1_w, self.n1_b, self.n2_w, self.n2_b]


class PackedLayer:
    """Padded device copies of one layer's weights (rebuilt from the real params each step)."""

    def __init__(self, d: int, ff: int, device):
        dp, ffp = rup(d, 64), rup(ff, 64)
        self.d, self.ff, self.dp, self.ffp = d, ff, dp, ffp
        z = lambda *s: torch.zeros(*s, device=device, dtype=torch.float32)  # noqa: E731
        self.W_in, self.b_in = z(3 * dp, dp), z(3 * dp)
        self.W_o, self.b_o = z(dp, dp), z(dp)
        self.W1, self.b1 = z(ffp, dp), z(ffp)
        self.W2, self.b2 = z(dp, ffp), z(dp)

    def jobs(self, p: LayerParams):
        """pack_padded_multi jobs refreshing the padded copies from the real parameters."""
        d, ff, dp, ffp = self.d, self.ff, self.dp, self.ffp
        return [(p.in_w, d, 3 * dp, dp, (dp, d), (dp, d), self.W_in, dp),
                (p.in_b, 3 * d, 1, 3 * dp, (1, 1), (dp, d), self.b_in, 3 * dp),
                (p.out_w, d, dp, dp, (dp, d), (dp, d), self.W_o, dp),
                (p.out_b, d, 1, dp, (1, 1), (dp, d), self.b_o, dp),
                (p.l1_w, d, ffp, dp, (ffp, ff), (dp, d), self.W1, dp),
                (p.l1_b, ff, 1, ffp, (1, 1), (ffp, ff), self.b1, ffp),
                (p.l2_w, ff, dp, ffp, (dp, d), (ffp, ff), self.W2, ffp),
                (p.l2_b, d, 1, dp, (1, 1), (dp, d), self.b2, dp)]

    def pack(self, p: LayerParams):
        K.pack_padded_multi(self.jobs(p))


class EncoderLayerCtx:
    """Saved forward tensors of one layer; Pd is the [Np, Np] signed probability image, or for d <= 32
    (small_attn) the attention context (attn_small_ctx_floats: the row statistics the backward recomputes P
    from and a compact Q, K, V copy)."""
    __slots__ = ("X", "QKV", "Pd", "O", "Z1", "X1", "mean1", "rstd1", "Hd", "Z2", "mean2", "rstd2",
                 "seeds")


# weight gradients on the 16-deep-K 128x128 tile (-1 % step time, A/B on one box)
_DEEP_WGRAD = True


def deep_wgrad() -> bool:
    return _DEEP_WGRAD


# Gradient work off the backward's critical path (weight, bias and LayerNorm-parameter gradients)
# runs on a second HIP stream, overlapping the dX chain; set_overlap(False) serialises it.
_OVERLAP = [True]
_SIDE: Dict[int, "torch.cuda.Stream"] = {}


def set_overlap(on: bool) -> bool:
    """Enable/disable the side stream (bench.py serialises its per-kernel timing pass, where
    concurrent kernels would inflate each other's event times); returns the previous setting."""
    prev = _OVERLAP[0]
    _OVERLAP[0] = bool(on)
    return prev


def side_stream(dev: torch.device) -> "torch.cuda.Stream":
    """The per-device side stream (created on first use).  It only overlaps the main stream when
    it has a hardware queue of its own: with RCCL's streams in the process, HIP's default 4 queues
    put it on the main stream's queue (the 1 ms/step of overlap at C4 was lost, whatever the
    creation order); u2gnn_hip.ensure_hw_queues raises the count to 8 at import."""
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(device=dev)
    return s



# The side stream pays only when the layer's kernels fill the chip: at C4 (Np*dp = 1.9M) it saves
# 0.31 ms of a 3.27 ms step; at C5 (U2GNN-UnSup REDDIT, d = 4: Np*dp = 0.13M, ~2-10 us kernels) the
# cross-stream hand-offs cost more than the overlap gains (1.116 vs 1.19-1.28 ms/step, one session,
# profiles/r02/r2i_graph_knobs.txt).
SIDE_MIN_ELEMS = int(os.environ.get("U2GNN_SIDE_MIN_ELEMS", 1 << 20))   # (env: A/B experiments only)


def fused_ln(dp: int, prec: str) -> bool:
    """LayerNorm forward inside the bias-dropout-residual GEMM epilogue: d <= 64 (one 64-column tile
    per row), matrix-core precisions (encoder_layer.cpp applies the same rule)."""
    return dp == 64 and prec != "fp32"


def ln_delta(prec: str) -> bool:
    """The attention backward's delta = rowsum(dO * O) from LayerNorm1's backward
    (layernorm_bwd_delta) in the matrix-core precisions; the fp32 parity path keeps its own rowdot
    launch, whose error does not grow with |X| (encoder_layer.cpp applies the same rule)."""
    return prec != "fp32"


def side_stream_pays(dims: "Dims") -> bool:
    return dims.Np * dims.dp >= SIDE_MIN_ELEMS


class OffPath:
    """Enqueue closures on the side stream after everything already issued on the current
    stream; tensors they read are record_stream'ed so the caching allocator cannot recycle
    them early.  join() makes the current stream wait for all of it.  enabled=False (or
    set_overlap(False)): everything runs on the current stream."""

    def __init__(self, dev: torch.device, enabled: bool = True):
        self.side = side_stream(dev) if enabled and _OVERLAP[0] and dev.type == "cuda" else None

    def run(self, fn, *uses: torch.Tensor):
        if self.side is None:
            fn()
            return
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            fn()
        for t in uses:
            t.record_stream(self.side)

    def join(self):
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)


BIG_TILE_BLOCKS = 768
# slab cap of the deep weight-gradient products (encoder_layer.cpp applies the same rule): at node-sized
# depths 8 slabs move half the bytes of 16 beside the main stream (C4 3.236 / 3.238 vs 3.251 / 3.260 ms;
# 12: 3.26, 4: 3.27); token-sized depths (neighbour mode, K = 82 K rows) keep 16 (8: 15.2 vs 13.9 ms).


def wgrad_split_cap(kd: int) -> int:
    return 8 if kd <= 8192 else 16


# Precision experiments (Python orchestration only): products (by role) that run plain bf16 when the
# layer runs bf16x3; tools/prec_probe.py fills ROLE_BF16 to measure each role's parity error.
ROLES = ("in_proj", "qk", "pv", "out_proj", "ffn1", "ffn2", "ffn2_dx", "ffn2_dw", "ffn1_dx", "ffn1_dw",
         "out_dx", "out_dw", "dv", "ds", "dq", "dk", "in_dx", "in_dw")
ROLE_BF16: set = set()
# precision "mixed" (experiment, not parity-grade): bf16x3 everywhere except the attention-backward
# products dS, dQ, dK on plain bf16 (u2gnn_hip.h U2GNN_LAYER_ATTN_BWD_BF16).  Joint error on C4
# batches (tools/prec_probe.py --mixed, profiles/r02/r2b_mixed_probe.log) 2.5e-4..4.0e-4 of the 1e-3
# bound, but the MUTAG L2T2 golden (d = 7) exceeds it; +4 % C4 step rate.  The forward products and
# the weight/input-gradient products are far outside the bound in plain bf16 (0.09..0.39: ReLU units
# flipping), so they stay bf16x3.
MIXED_BF16_ROLES = ("ds", "dq", "dk")
# Precision experiments (Python orchestration only): role -> precision overriding the layer's
# (tools/prec_train_probe.py measures train-mode parity per policy).
ROLE_PREC: Dict[str, str] = {}
# precision "fwd32": the forward products exact fp32 (so the forward's ReLU decisions carry fp32 rounding
# only), the backward bf16x3 (u2gnn_hip.h U2GNN_LAYER_FWD_F32); precision "fwd6": the
# forward products on the three-plane bf16x6 split (fp32-accurate products at 6/16 of the bf16 MFMA rate instead
# of 1/16), the backward bf16x3 (U2GNN_LAYER_FWD_X6); precision "fwdh": the forward products on the two-plane fp16
# split f16x3 (~2^-21 per product at the bf16x3 rate), the backward bf16x3 (U2GNN_LAYER_FWD_H3)
FWD_ROLES = ("in_proj", "qk", "pv", "out_proj", "ffn1", "ffn2")


def _rp(role: str, prec: str) -> str:
    """Matrix-core precision of one product (role) of a layer running at `prec`."""
    if role in ROLE_PREC:
        return ROLE_PREC[role]
    if prec == "mixed":
        return "bf16" if role in MIXED_BF16_ROLES else "bf16x3"
    if prec == "fwd32":
        return "fp32" if role in FWD_ROLES else "bf16x3"
    if prec == "fwd6":
        return "bf16x6" if role in FWD_ROLES else "bf16x3"
    if prec == "fwdh":
        return "f16x3" if role in FWD_ROLES else "bf16x3"
    return "bf16" if (prec == "bf16x3" and role in ROLE_BF16) else prec


def _gemm_split(A, B, C, M, N, Kd, lda, ldb, ldc, trans_a=False, trans_b=False, alpha=1.0, accumulate=False,
                prec="fp32", rblk=None, cblk=None, target=448, flops=None, deep=False, clamp_a=False, target256=240,
                h3_exp=None):
    """C (+)= alpha * op(A) . op(B) with deterministic split-K: when the tile grid alone would
    leave most of the 256 CUs idle (skinny outputs with a deep node dimension: P.V, Pd^T.dO,
    dS.K, dS^T.Q, the weight gradients, dH.W1, dQKV.W_in), the depth is cut into fp32 slabs
    (>= 4 K-tiles each, ~target workgroups) and one streaming pass sums them into C — applying
    alpha, accumulation and an optional padded->real block map (rblk, cblk).  clamp_a: A is the
    signed probability image (read as Pd).  h3_exp: the f16x3 operand pre-scales (kernels.gemm)."""
    bk = 16 if prec == "fp32" else 32
    # tiny: an accumulating product of <= 16 tiles and <= 16 K steps (C2's dX += dQKV W_in) as one short launch
    tiny = accumulate and Kd <= 512 and (M // 64) * (N // 64) <= 16
    if (prec != "fp32" and not deep and rblk is None and Kd <= 2048 and M % 64 == 0
            and N % 64 == 0 and ((M // 64) * (N // 64) >= 256 or tiny)):
        # shallow K (dH.W1, dQKV.W_in: K = ff, 3d) with enough 64x64 tiles to fill the chip: no
        # split, C (+)= alpha acc straight from the epilogue -- no slabs, no reduce pass
        K.gemm(A, B, C, M, N, Kd, lda, ldb, ldc, trans_a=trans_a, trans_b=trans_b, alpha=alpha,
               epilogue=E.EPI_ACCUM if accumulate else E.EPI_STORE, precision=prec,
               tile=256 if (M % 256 == 0 and N % 128 == 0 and (M // 256) * (N // 128) >= BIG_TILE_BLOCKS) else 64,
               flops=flops, clamp_a=clamp_a, h3_exp=h3_exp)
        return
    if prec != "fp32" and M % 256 == 0 and N % 128 == 0 and (M // 256) * (N // 128) >= 32:
        # 256x128 blocks (8 waves, one block per CU): the skinny attention products
        t, tiles, target = 256, (M // 256) * (N // 128), target256
    else:
        t = 128 if (M % 128 == 0 and N % 128 == 0) else 64
        tiles = (M // t) * (N // t)
    split = max(1, min(target // max(tiles, 1), Kd // (4 * bk)))
    if deep and _DEEP_WGRAD and prec != "fp32" and t == 128:
        # weight gradients (a few dozen 128x128 output tiles, K = Np): the 16-deep K step runs 3
        # blocks per CU; <= 16 slabs keeps the reduce pass short
        t, split = 129, max(1, min(wgrad_split_cap(Kd), target // max(tiles, 1)))
    mapped = rblk is not None
    if split == 1 and not mapped:
        K.gemm(A, B, C, M, N, Kd, lda, ldb, ldc, trans_a=trans_a, trans_b=trans_b, alpha=alpha,
               epilogue=E.EPI_ACCUM if accumulate else E.EPI_STORE, precision=prec, tile=t, flops=flops,
               clamp_a=clamp_a, h3_exp=h3_exp)
        return
    slabs = torch.empty(split, M, N, device=C.device, dtype=torch.float32)
    K.gemm(A, B, slabs, M, N, Kd, lda, ldb, N, trans_a=trans_a, trans_b=trans_b, split_k=split, slab_stride=M * N,
           precision=prec, tile=t, flops=flops, clamp_a=clamp_a, h3_exp=h3_exp)
    K.slab_reduce(slabs, split, M * N, M, N, N, rblk or (M, M), cblk or (N, N), C, ldc, alpha=alpha,
                  accumulate=accumulate)


def _wgrad(dY, ld_dy, X, ld_x, m_pad, n_pad, rows_pad, dst, rblk, cblk, prec, n_real):
    """dst(real) = unpack(dY^T X) with dY [rows_pad, m_pad] (ld_dy), X [rows_pad, n_pad] (ld_x)."""
    _gemm_split(dY, X, dst, m_pad, n_pad, rows_pad, ld_dy, ld_x, dst.shape[-1] if dst.dim() > 1 else dst.numel(),
                trans_a=True, prec=prec, rblk=rblk, cblk=cblk, flops=2.0 * dst.numel() * n_real, deep=True)


def _bias_grad(dY, rows, cols_pad, ld, cblk, out):
    ws = torch.empty(max(4, K.colstat_ws_floats(rows, cols_pad)), device=dY.device, dtype=torch.float32)
    K.colsum(dY, rows, cols_pad, ld, cblk, out, ws)


def in_bias_grad(dQKV, Np, dp, d, out):
    """in_proj_bias gradient: column sums of dQKV's Q and V thirds; the K third is exactly zero (a softmax row
    is invariant to a constant added to its scores: sum_j dK_j = sum_i Q_i sum_j dS_ij = 0), written as the
    column sum of zero rows.  Mirrors encoder_layer.cpp (same launches, same bits)."""
    _bias_grad(dQKV, Np, dp, 3 * dp, (dp, d), out[:d])
    _bias_grad(dQKV[:, dp:], 0, dp, 3 * dp, (dp, d), out[d:2 * d])
    _bias_grad(dQKV[:, 2 * dp:], Np, dp, 3 * dp, (dp, d), out[2 * d:])


def _gemm_nodes_k(A, B, C, M, N, Kd, lda, ldb, ldc, trans_a=False, alpha=1.0, prec="fp32", flops=None,
                  clamp_a=False, grouped=False, h3_exp=None):
    """The skinny attention products whose depth is the node dimension (N = dp, K = Np).  grouped: dQ / dK,
    which the native executor issues as one grouped launch -- half the 256x128 block target each
    (encoder_layer.cpp gemm_split), so both paths cut the same split-K slabs."""
    _gemm_split(A, B, C, M, N, Kd, lda, ldb, ldc, trans_a=trans_a, alpha=alpha, prec=prec, flops=flops,
                clamp_a=clamp_a, target256=120 if grouped else 240, h3_exp=h3_exp)


def ffn2_split(dp: int, mfma: bool, Np: int, ffp: int) -> int:
    """Split-K depth of FFN2 in the matrix-core precisions (encoder_layer.cpp ffn2_split), dp <= 256: with
    fewer than 128 output tiles of 64x64, ~256 blocks of >= 4 K steps, finished by slab_bias_drop_resid_ln
    (bias, dropout, residual and LayerNorm2)."""
    tiles = (Np // 64) * (dp // 64)
    if not mfma or dp > 256 or tiles >= 128:
        return 1
    return max(1, min(256 // tiles, ffp // 128))


def qk_tile(Np: int) -> int:
    """Tile of the S = Q K^T product (encoder_layer.cpp qk_tile): 256x128 blocks unless they would leave
    most CUs idle (C5's Np = 2048: 128 blocks), then 128x128 (same per-element sums, same bits)."""
    return 256 if Np % 256 == 0 and (Np // 256) * (Np // 128) >= 256 else 128


SMALL_ATTN_MAX_D = 32


def small_attn(d: int) -> bool:
    """Node attention on the vector ALUs, flash-style (u2gnn_attn_small_*): feature widths d <= 32 in every
    precision -- the matrix-core products would be >= 50 % padding (dp = 64) and the N x N images pure
    overhead (encoder_layer.cpp small_attn applies the same rule)."""
    return d <= SMALL_ATTN_MAX_D


def mid_tail(d: int, dp: int, Np: int) -> bool:
    """The forward tail (a3.3 + a3.4) of a mid-width layer with few rows as one row-block kernel + the slab
    LayerNorm (u2gnn_layer_tail_mid_fwd; encoder_layer.cpp mid_tail applies the same rule)."""
    return d > SMALL_ATTN_MAX_D and dp <= 256 and Np <= 512


FUSED_MIN_NP = 1024   # encoder_layer.cpp kFusedMinNp


def fused_attn(dp: int, prec_qk: str, prec_pv: str, Np: int = FUSED_MIN_NP) -> bool:
    """Node-axis attention forward through the fused softmax.P.V kernel: Q K^T with the row-statistics epilogue
    (bf16, bf16x3, bf16x6 or f16x3) and P.V in bf16 / bf16x3 / f16x3, dp <= 384, Np >= FUSED_MIN_NP
    (encoder_layer.cpp fused_attn: fewer rows run the three-pass form; the fwd6 policy keeps the three-pass form,
    the kernel's bf16x6 P.V is a tested capability, measured no faster)."""
    return prec_qk != "fp32" and prec_pv in ("bf16", "bf16x3", "f16x3") and dp <= 384 and Np >= FUSED_MIN_NP


def _attn_split(Q, Kt, V, N, Np, dp, pd, seeds, prec, att, dev):
    """a3.2 as three passes (fp32 parity path, dp > 384): S = Q K^T, softmax + dropout into the image,
    split-K P.V."""
    f32 = torch.float32
    S = torch.empty(Np, Np, device=dev, dtype=f32)
    K.gemm(Q, Kt, S, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True, precision=_rp("qk", prec), flops=att,
           tile=256 if (_rp("qk", prec) != "fp32" and Np % 256 == 0) else 0)
    # one [Np, Np] image: with dropout the signed one (P/(1-p) where kept, -P where dropped), which
    # P.V and dP^T.dO read as Pd (negatives staged as 0) and the dS epilogue reads as P and keep
    Pd = torch.empty(Np, Np, device=dev, dtype=f32)
    K.attn_softmax_fwd(S, Np, None if pd > 0 else Pd, Pd, Np, N, Np, N, Np, pd, seeds.get(SITE_ATTN, 0))
    del S
    O = torch.empty(Np, dp, device=dev, dtype=f32)
    _gemm_nodes_k(Pd, V, O, Np, dp, Np, Np, 3 * dp, dp, prec=_rp("pv", prec), flops=att, clamp_a=pd > 0,
                  h3_exp=(K.h3_prob_exp(pd), K.H3_EXP) if _rp("pv", prec) == "f16x3" else None)
    # (f16x3: the probability image's pre-scale, encoder_layer.cpp h3_prob_exp)
    return Pd, O


def encoder_layer_forward(X: torch.Tensor, w: PackedLayer, p: LayerParams, dims: Dims, train: bool,
                          seeds: Dict[int, int], need_ctx: bool, prec: str = "fp32",
                          p_drop: float = 0.5) -> (torch.Tensor, Optional[EncoderLayerCtx]):
    """One torch TransformerEncoderLayer(d, nhead=1, ff, dropout=0.5) forward, post-LN, on the
    slot-0 rows X [Np, dp] (pytorch_U2GNN_Sup.py:19-21,35)."""
    N, Np, d, dp, ff, ffp = dims.N, dims.Np, dims.d, dims.dp, dims.ff, dims.ffp
    pd = p_drop if train else 0.0
    att = 2.0 * N * N * d          # algorithmic FLOPs of one attention product (real N, d)
    dev = X.device
    f32 = torch.float32
    small = small_attn(d)
    fused = not small and fused_attn(dp, _rp("qk", prec), _rp("pv", prec), Np)
    QKV = QKV2 = None
    if not small:   # (the small-width attention projects into its own compact context)
        QKV = torch.empty(Np, 3 * dp, device=dev, dtype=f32)
        # x2 copy of V for the fused P.V (bf16x6 P.V reads the fp32 output itself)
        # (f16x3: fp16 planes of 2^U2GNN_H3_X2_EXP V in the same layout)
        QKV2 = torch.empty(Np, 6 * dp, device=dev, dtype=torch.bfloat16) if fused and _rp("pv", prec) != "bf16x6" else None
        K.gemm(X, w.W_in, QKV, Np, 3 * dp, dp, dp, dp, 3 * dp, trans_b=True, epilogue=E.EPI_BIAS, bias=w.b_in,
               alpha=1.0 / math.sqrt(d), scale_cols=dp, precision=_rp("in_proj", prec), flops=6.0 * N * d * d,
               tile=256 if (_rp("in_proj", prec) != "fp32" and Np % 256 == 0 and (Np // 256) * (3 * dp // 128) >= BIG_TILE_BLOCKS) else 0,
               Cx2=QKV2, ldcx2=6 * dp, cx2_col0=2 * dp)
        Q, Kt, V = QKV[:, :dp], QKV[:, dp:2 * dp], QKV[:, 2 * dp:]
    if small:
        # d <= 32: the whole layer on the vector ALUs (issued below with the tail: encoder_layer.cpp layer_fwd,
        # launch for launch); the row statistics and a compact Q, K, V take the images' place in the context
        O = torch.empty(Np, dp, device=dev, dtype=f32)
        Pd = torch.empty(K.attn_small_ctx_floats(Np, d), device=dev, dtype=f32)
    elif fused:
        # S = Q K^T written straight into the image buffer, with the softmax row partials of each 64-column
        # group from the GEMM epilogue; one fused softmax -> dropout -> P.V pass then overwrites S with the
        # signed image and forms O (attn_fused.hip; encoder_layer.cpp layer_fwd, launch for launch)
        Pd = torch.empty(Np, Np, device=dev, dtype=f32)
        rowpart = torch.empty(Np, 2 * (Np // 32), device=dev, dtype=f32)
        K.gemm(Q, Kt, Pd, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True, epilogue=E.EPI_STORE_ROWSTAT,
               rowpart=rowpart, n_valid=N, precision=_rp("qk", prec), flops=att, tile=qk_tile(Np))
        ws = torch.empty(K.attn_softmax_pv_ws_floats(N, Np, dp), device=dev, dtype=f32)
        O = torch.empty(Np, dp, device=dev, dtype=f32)
        x6 = _rp("pv", prec) == "bf16x6"
        K.attn_softmax_pv(Pd, Np, rowpart, Np // 64, QKV if x6 else QKV2, 3 * dp if x6 else 6 * dp, dp, Pd, Np, O, dp,
                          ws, N, Np, pd, seeds.get(SITE_ATTN, 0), precision=_rp("pv", prec))
        del QKV2, rowpart, ws
    else:
        Pd, O = _attn_split(Q, Kt, V, N, Np, dp, pd, seeds, prec, att, dev)
    Z1 = torch.empty(Np, dp, device=dev, dtype=f32)
    X1 = torch.empty(Np, dp, device=dev, dtype=f32)
    mean1 = torch.empty(Np, device=dev, dtype=f32)
    rstd1 = torch.empty(Np, device=dev, dtype=f32)
    Hd = torch.empty(Np, ffp, device=dev, dtype=f32)
    Z2 = torch.empty(Np, dp, device=dev, dtype=f32)
    X2 = torch.empty(Np, dp, device=dev, dtype=f32)
    mean2 = torch.empty(Np, device=dev, dtype=f32)
    rstd2 = torch.empty(Np, device=dev, dtype=f32)
    if small:
        # in-projection, attention, a3.3 + a3.4 on the vector ALUs: 2 or 3 launches (encoder_layer.cpp layer_fwd)
        K.layer_small_fwd(N, Np, d, dp, ff, ffp, pd, (seeds.get(SITE_DROP1, 0), seeds.get(SITE_DROPFF, 0),
                          seeds.get(SITE_DROP2, 0)), seeds.get(SITE_ATTN, 0), w.W_in, w.b_in, Pd, W_o=w.W_o,
                          b_o=w.b_o, n1_w=p.n1_w, n1_b=p.n1_b, W1=w.W1, b1=w.b1, W2=w.W2, b2=w.b2, n2_w=p.n2_w,
                          n2_b=p.n2_b, O=O, X=X, Z1=Z1, X1=X1, mean1=mean1, rstd1=rstd1, Hd=Hd, Z2=Z2, X2=X2,
                          mean2=mean2, rstd2=rstd2)
    elif mid_tail(d, dp, Np):
        # a3.3 + a3.4 in two launches: out-projection .. FFN2 partials per row block and hidden chunk, then the slab
        # LayerNorm2 (mid_layer.hip; encoder_layer.cpp layer_fwd, launch for launch)
        ws = torch.empty(K.layer_tail_mid_ws_floats(Np, dp, ffp), device=dev, dtype=f32)
        K.layer_tail_mid_fwd(N, Np, d, dp, ff, ffp, pd, (seeds.get(SITE_DROP1, 0), seeds.get(SITE_DROPFF, 0),
                             seeds.get(SITE_DROP2, 0)), ws, W_o=w.W_o, b_o=w.b_o, n1_w=p.n1_w, n1_b=p.n1_b, W1=w.W1,
                             b1=w.b1, W2=w.W2, b2=w.b2, n2_w=p.n2_w, n2_b=p.n2_b, O=O, X=X, Z1=Z1, X1=X1, mean1=mean1,
                             rstd1=rstd1, Hd=Hd, Z2=Z2, X2=X2, mean2=mean2, rstd2=rstd2)
        del ws
    else:
        fuse = fused_ln(dp, _rp("out_proj", prec))   # LayerNorm in the GEMM epilogue when a 64-column tile holds whole rows
        K.gemm(O, w.W_o, Z1, Np, dp, dp, dp, dp, dp, trans_b=True,
               epilogue=E.EPI_BIAS_DROP_RESID_LN if fuse else E.EPI_BIAS_DROP_RESID, bias=w.b_o,
               aux0=X, ld_aux=dp, p_drop=pd, seed=seeds.get(SITE_DROP1, 0), precision=_rp("out_proj", prec),
               flops=2.0 * N * d * d, ln=(p.n1_w, p.n1_b, X1, dp, mean1, rstd1, d, N, 1e-5) if fuse else None)
        if not fuse:
            K.layernorm_fwd(Z1, dp, p.n1_w, p.n1_b, X1, dp, mean1, rstd1, N, Np, d, dp)
        K.gemm(X1, w.W1, Hd, Np, ffp, dp, dp, dp, ffp, trans_b=True, epilogue=E.EPI_BIAS_RELU_DROP, bias=w.b1,
               p_drop=pd, seed=seeds.get(SITE_DROPFF, 0), precision=_rp("ffn1", prec), flops=2.0 * N * d * ff)
        # (dp = 64: the out-projection's fused-LayerNorm rule decides, as in round 3)
        f2 = ffn2_split(dp, fuse if dp == 64 else _rp("ffn2", prec) != "fp32", Np, ffp)
        if f2 > 1:   # split-K slabs + the bias / dropout / residual / LayerNorm pass (encoder_layer.cpp layer_fwd)
            slabs = torch.empty(f2, Np, dp, device=dev, dtype=f32)
            K.gemm(Hd, w.W2, slabs, Np, dp, ffp, ffp, ffp, dp, trans_b=True, split_k=f2, slab_stride=Np * dp,
                   precision=_rp("ffn2", prec), flops=2.0 * N * d * ff, tile=64)
            K.slab_bias_drop_resid_ln(slabs, f2, Np * dp, w.b2, X1, pd, seeds.get(SITE_DROP2, 0), Z2, p.n2_w, p.n2_b,
                                      X2, mean2, rstd2, d, N, Np)
            del slabs
        else:
            K.gemm(Hd, w.W2, Z2, Np, dp, ffp, ffp, ffp, dp, trans_b=True,
                   epilogue=E.EPI_BIAS_DROP_RESID_LN if fuse else E.EPI_BIAS_DROP_RESID, bias=w.b2,
                   aux0=X1, ld_aux=dp, p_drop=pd, seed=seeds.get(SITE_DROP2, 0), precision=_rp("ffn2", prec),
                   flops=2.0 * N * d * ff, ln=(p.n2_w, p.n2_b, X2, dp, mean2, rstd2, d, N, 1e-5) if fuse else None)
        if not fuse and f2 <= 1:
            K.layernorm_fwd(Z2, dp, p.n2_w, p.n2_b, X2, dp, mean2, rstd2, N, Np, d, dp)
    ctx = None
    if need_ctx:
        ctx = EncoderLayerCtx()
        ctx.X, ctx.QKV, ctx.Pd, ctx.O = X, QKV, Pd, O
        ctx.Z1, ctx.X1, ctx.mean1, ctx.rstd1, ctx.Hd = Z1, X1, mean1, rstd1, Hd
        ctx.Z2, ctx.mean2, ctx.rstd2 = Z2, mean2, rstd2
        ctx.seeds = (pd, dict(seeds))
    return X2, ctx


def encoder_layer_backward(dX2: torch.Tensor, ctx: EncoderLayerCtx, w: PackedLayer, p: LayerParams,
                           g: LayerParams, dims: Dims, prec: str = "fp32",
                           off: Optional[OffPath] = None, need_dx: bool = True) -> Optional[torch.Tensor]:
    """Backward of encoder_layer_forward (``need_dx=False``: the input gradient is not wanted,
    its in-projection GEMM is skipped and None is returned).  Writes the real-shaped parameter gradients into
    ``g`` (tensors shaped like the params) and returns dX [Np, dp].  Parameter-gradient work is
    enqueued on ``off``'s side stream (joined here unless the caller passes its own OffPath)."""
    N, Np, d, dp, ff, ffp = dims.N, dims.Np, dims.d, dims.dp, dims.ff, dims.ffp
    pd, seeds = ctx.seeds
    att = 2.0 * N * N * d
    dev = dX2.device
    f32 = torch.float32
    own = off is None
    if own:
        off = OffPath(dev)
    ws = torch.empty(K.colstat_ws_floats(N, dp), device=dev, dtype=f32)
    use_ln_delta = ln_delta(_rp("ds", prec))
    if small_attn(d):
        # the row-local tail in one launch: dX1, dF, dH, dX, dA, dO and delta (encoder_layer.cpp layer_bwd); the
        # parameter gradients on the side stream in the matrix-core branch's order
        dX1, dF, dA, dO, dX = (torch.empty(Np, dp, device=dev, dtype=f32) for _ in range(5))
        dH = torch.empty(Np, ffp, device=dev, dtype=f32)
        delta = torch.empty(Np, device=dev, dtype=f32)
        # the tail backward and the attention backward (dQKV; dX += dQKV W_in when the input gradient is wanted)
        small_dqkv = torch.empty(Np, 3 * dp, device=dev, dtype=f32)
        ws_a = torch.empty(K.attn_small_ws_floats(N, Np, d), device=dev, dtype=f32)
        K.layer_small_bwd(N, Np, d, dp, ff, ffp, pd, (seeds.get(SITE_DROP1, 0), seeds.get(SITE_DROPFF, 0),
                          seeds.get(SITE_DROP2, 0)), seeds.get(SITE_ATTN, 0), w.W_in, ctx.Pd, small_dqkv, need_dx,
                          ws_a, W_o=w.W_o, b_o=w.b_o, n1_w=p.n1_w, n1_b=p.n1_b, W1=w.W1, b1=w.b1, W2=w.W2, b2=w.b2,
                          n2_w=p.n2_w, n2_b=p.n2_b, O=ctx.O, Z1=ctx.Z1, X1=ctx.X1, mean1=ctx.mean1, rstd1=ctx.rstd1,
                          Hd=ctx.Hd, Z2=ctx.Z2, mean2=ctx.mean2, rstd2=ctx.rstd2, dX2=dX2, dX1=dX1, dF=dF, dH=dH,
                          dX=dX, dA=dA, dO=dO, delta=delta)
        del ws_a
        off.run(lambda: K.layernorm_bwd_params(dX2, dp, ctx.Z2, dp, ctx.mean2, ctx.rstd2, dF, dp, N, d, dp, ws, g.n2_w,
                                               g.n2_b, g.l2_b), dX2, ctx.Z2, ctx.mean2, ctx.rstd2, dF, ws)
        off.run(lambda: _wgrad(dF, dp, ctx.Hd, ffp, dp, ffp, Np, g.l2_w, (dp, d), (ffp, ff), _rp("ffn2_dw", prec), N),
                dF, ctx.Hd)

        def ffn1_grads_t(dH=dH):
            _wgrad(dH, ffp, ctx.X1, dp, ffp, dp, Np, g.l1_w, (ffp, ff), (dp, d), _rp("ffn1_dw", prec), N)
            _bias_grad(dH, Np, ffp, ffp, (ffp, ff), g.l1_b)
        off.run(ffn1_grads_t, dH, ctx.X1)
        off.run(lambda: K.layernorm_bwd_params(dX1, dp, ctx.Z1, dp, ctx.mean1, ctx.rstd1, dA, dp, N, d, dp, ws, g.n1_w,
                                               g.n1_b, g.out_b), dX1, ctx.Z1, ctx.mean1, ctx.rstd1, dA)
        off.run(lambda: _wgrad(dA, dp, ctx.O, dp, dp, dp, Np, g.out_w, (dp, d), (dp, d), _rp("out_dw", prec), N), dA, ctx.O)
        del dH, dF, dX1, dA
        use_ln_delta = True   # delta from the tail kernel
    else:
        # LN2 backward -> dX1 (residual branch), dF (dropout2 branch); norm2 + linear2.bias grads
        dX1 = torch.empty(Np, dp, device=dev, dtype=f32)
        dF = torch.empty(Np, dp, device=dev, dtype=f32)
        K.layernorm_bwd(dX2, dp, ctx.Z2, dp, ctx.mean2, ctx.rstd2, p.n2_w, dX1, dp, dF, dp, pd,
                        seeds.get(SITE_DROP2, 0), N, Np, d, dp)
        off.run(lambda: K.layernorm_bwd_params(dX2, dp, ctx.Z2, dp, ctx.mean2, ctx.rstd2, dF, dp, N, d, dp, ws, g.n2_w,
                                               g.n2_b, g.l2_b), dX2, ctx.Z2, ctx.mean2, ctx.rstd2, dF, ws)
        # FFN: Z2 = X1 + drop(Hd W2^T + b2), Hd = drop(relu(X1 W1^T + b1))
        dH = torch.empty(Np, ffp, device=dev, dtype=f32)
        K.gemm(dF, w.W2, dH, Np, ffp, dp, dp, ffp, ffp, epilogue=E.EPI_RELU_DROP_BWD, aux0=ctx.Hd, ld_aux=ffp,
               p_drop=pd, precision=_rp("ffn2_dx", prec), flops=2.0 * N * d * ff)
        off.run(lambda: _wgrad(dF, dp, ctx.Hd, ffp, dp, ffp, Np, g.l2_w, (dp, d), (ffp, ff), _rp("ffn2_dw", prec), N), dF, ctx.Hd)
        _gemm_split(dH, w.W1, dX1, Np, dp, ffp, ffp, dp, dp, accumulate=True, prec=_rp("ffn1_dx", prec), flops=2.0 * N * d * ff)

        def ffn1_grads(dH=dH):
            _wgrad(dH, ffp, ctx.X1, dp, ffp, dp, Np, g.l1_w, (ffp, ff), (dp, d), _rp("ffn1_dw", prec), N)
            _bias_grad(dH, Np, ffp, ffp, (ffp, ff), g.l1_b)
        off.run(ffn1_grads, dH, ctx.X1)
        del dH, dF
        # LN1 backward -> dX (residual), dA (dropout1 branch)
        dX = torch.empty(Np, dp, device=dev, dtype=f32)
        dA = torch.empty(Np, dp, device=dev, dtype=f32)
        if use_ln_delta:   # LayerNorm1's backward also forms the attention backward's delta = rowsum(dO * O)
            delta = torch.empty(Np, device=dev, dtype=f32)
            K.layernorm_bwd_delta(dX1, dp, ctx.Z1, dp, ctx.mean1, ctx.rstd1, p.n1_w, dX, dp, dA, dp, pd,
                                  seeds.get(SITE_DROP1, 0), N, Np, d, dp, ctx.X, dp, w.b_o, delta)
        else:
            K.layernorm_bwd(dX1, dp, ctx.Z1, dp, ctx.mean1, ctx.rstd1, p.n1_w, dX, dp, dA, dp, pd,
                            seeds.get(SITE_DROP1, 0), N, Np, d, dp)
        off.run(lambda: K.layernorm_bwd_params(dX1, dp, ctx.Z1, dp, ctx.mean1, ctx.rstd1, dA, dp, N, d, dp, ws, g.n1_w,
                                               g.n1_b, g.out_b), dX1, ctx.Z1, ctx.mean1, ctx.rstd1, dA)
        del dX1
        # out-projection
        dO = torch.empty(Np, dp, device=dev, dtype=f32)
        K.gemm(dA, w.W_o, dO, Np, dp, dp, dp, dp, dp, precision=_rp("out_dx", prec), flops=2.0 * N * d * d)
        off.run(lambda: _wgrad(dA, dp, ctx.O, dp, dp, dp, Np, g.out_w, (dp, d), (dp, d), _rp("out_dw", prec), N), dA, ctx.O)
        del dA
    # attention core
    QKV = ctx.QKV
    if not use_ln_delta:
        delta = torch.empty(Np, device=dev, dtype=f32)
        K.rowdot(dO, dp, ctx.O, dp, delta, Np, dp)
    if small_attn(d):
        # d <= 32: dQ, dK, dV (P recomputed from the saved context) and dX += dQKV W_in, run with the tail above
        dQKV = small_dqkv
        del dO
    else:
        dQKV = _attn_bwd_products(ctx, dO, delta, N, Np, d, dp, pd, att, prec, dev)
    _in_proj_backward(dQKV, dX, ctx, w, g, N, Np, d, dp, prec, off, need_dx)
    if own:
        off.join()
    return dX if need_dx else None


def _attn_bwd_products(ctx, dO, delta, N, Np, d, dp, pd, att, prec, dev):
    """dS (matrix cores, from the signed image), then dV = Pd^T dO, dQ = dS K / sqrt(d), dK = dS^T Q."""
    f32 = torch.float32
    QKV = ctx.QKV
    Q, Kt, V = QKV[:, :dp], QKV[:, dp:2 * dp], QKV[:, 2 * dp:]
    dS = torch.empty(Np, Np, device=dev, dtype=f32)
    K.gemm(dO, V, dS, Np, Np, dp, dp, 3 * dp, Np, trans_b=True, epilogue=E.EPI_ATTN_DS_SIGNED, aux0=ctx.Pd,
           p_drop=pd, rowvec=delta, ld_aux=Np, precision=_rp("ds", prec), flops=att)
    dQKV = torch.empty(Np, 3 * dp, device=dev, dtype=f32)
    _gemm_nodes_k(ctx.Pd, dO, dQKV[:, 2 * dp:], Np, dp, Np, Np, dp, 3 * dp, trans_a=True, prec=_rp("dv", prec), flops=att,
                  clamp_a=pd > 0)
    _gemm_nodes_k(dS, Kt, dQKV[:, :dp], Np, dp, Np, Np, 3 * dp, 3 * dp, alpha=1.0 / math.sqrt(d), prec=_rp("dq", prec),
                  flops=att, grouped=True)
    _gemm_nodes_k(dS, Q, dQKV[:, dp:2 * dp], Np, dp, Np, Np, 3 * dp, 3 * dp, trans_a=True, prec=_rp("dk", prec), flops=att,
                  grouped=True)
    del dS, dO
    return dQKV


def _in_proj_backward(dQKV, dX, ctx, w, g, N, Np, d, dp, prec, off, need_dx):
    """dX += dQKV W_in (skipped when the input gradient is not wanted); the in-projection's weight and bias
    gradients (on the side stream unless this is the last layer of the backward)."""
    if need_dx and not small_attn(d):   # (the small-width attention backward adds dQKV W_in itself)
        _gemm_split(dQKV, w.W_in, dX, Np, dp, 3 * dp, 3 * dp, dp, dp, accumulate=True, prec=_rp("in_dx", prec),
                    flops=6.0 * N * d * d)

    def in_proj_grads(dQKV=dQKV):
        _wgrad(dQKV, 3 * dp, ctx.X, dp, 3 * dp, dp, Np, g.in_w, (dp, d), (dp, d), _rp("in_dw", prec), N)
        in_bias_grad(dQKV, Np, dp, d, g.in_b)
    if need_dx:
        off.run(in_proj_grads, dQKV, ctx.X)
    else:   # the last layer of the backward: nothing left on this stream to overlap, skip the hand-off
        in_proj_grads()
