"""Per-kernel numerics of libu2gnn_hip.so against plain torch fp32 references (GPU)."""
import ctypes
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import _lib  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402

DEV = "cuda"


def rel_err(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _mk(*s, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*s, generator=g).to(DEV)


@pytest.mark.parametrize("tile", [64, 128])
@pytest.mark.parametrize("layout", ["NT", "NN", "TN"])
def test_gemm_layouts_exact_fp32(tile, layout):
    M, N, Kd = 256, 384, 192
    ta, tb = layout[0] == "T", layout[1] == "T"
    A = _mk(Kd, M, seed=1) if ta else _mk(M, Kd, seed=1)
    B = _mk(N, Kd, seed=2) if tb else _mk(Kd, N, seed=2)
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, A.shape[1], B.shape[1], N, trans_a=ta, trans_b=tb, tile=tile)
    ref = (A.t() if ta else A).double() @ (B.t() if tb else B).double()
    assert rel_err(C.double(), ref) < 1e-5


@pytest.mark.parametrize("prec,tol", [("bf16x3", 3e-5), ("bf16", 2e-2)])
@pytest.mark.parametrize("tile", [64, 128, 256, 129])
@pytest.mark.parametrize("layout", ["NT", "NN", "TN"])
def test_gemm_split_bf16_layouts(prec, tol, tile, layout):
    M, N, Kd = 512, 384, 320
    ta, tb = layout[0] == "T", layout[1] == "T"
    A = _mk(Kd, M, seed=11) if ta else _mk(M, Kd, seed=11)
    B = _mk(N, Kd, seed=12) if tb else _mk(Kd, N, seed=12)
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, A.shape[1], B.shape[1], N, trans_a=ta, trans_b=tb, tile=tile, precision=prec)
    ref = (A.t() if ta else A).double() @ (B.t() if tb else B).double()
    assert rel_err(C.double(), ref) < tol


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
def test_gemm_split_bf16_identity_and_epilogue(prec):
    M = N = Kd = 128
    A = torch.eye(M, device=DEV)
    B = (torch.arange(Kd * N, device=DEV, dtype=torch.float32).view(Kd, N) % 251) / 8.0   # exact in bf16
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, Kd, N, N, precision=prec)
    assert torch.equal(C, B)
    Bt = B.t().contiguous()
    P, Pd, dl = torch.rand(M, N, device=DEV), torch.rand(M, N, device=DEV), _mk(M, seed=9)
    K.gemm(A, Bt, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ATTN_DS, aux0=P, aux1=Pd, rowvec=dl,
           ld_aux=N, precision=prec)
    assert rel_err(C, Pd * B - P * dl[:, None]) < 1e-6


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C/D map."""
    M = N = Kd = 128
    A = torch.eye(M, device=DEV)
    B = torch.arange(Kd * N, device=DEV, dtype=torch.float32).view(Kd, N) / 1000.0
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, Kd, N, N)
    assert torch.equal(C, B)


def test_gemm_split_k_slabs_and_views():
    M, N, Kd = 128, 192, 1024
    A = _mk(Kd, M, seed=3)     # trans_a
    B = _mk(Kd, 3 * N, seed=4)[:, N:2 * N]   # column-slice view, ld 3N
    slabs = torch.empty(4, M, N, device=DEV)
    K.gemm(A, B, slabs, M, N, Kd, M, 3 * N, N, trans_a=True, split_k=4, slab_stride=M * N, tile=64)
    out = torch.empty(M, N, device=DEV)
    K.slab_reduce(slabs, 4, M * N, M, N, N, (M, M), (N, N), out, N)
    ref = A.t().double() @ B.double()
    assert rel_err(out.double(), ref) < 1e-5


@pytest.mark.parametrize("prec,Kd,split,tile", [("fp32", 208, 5, 128), ("fp32", 64, 8, 128), ("bf16x3", 352, 4, 128),
                                                ("bf16x3", 96, 8, 128), ("bf16x3", 352, 4, 256), ("bf16", 96, 8, 256),
                                                ("bf16x3", 336, 5, 129)])
def test_gemm_ragged_and_empty_splits(prec, Kd, split, tile):
    """split z covers [z*Kc, min((z+1)*Kc, K)); trailing splits may be short or empty (zero slab)."""
    M, N = 256, 128
    A, B = _mk(Kd, M, seed=31), _mk(Kd, N, seed=32)
    slabs = torch.full((split, M, N), float("nan"), device=DEV)
    K.gemm(A, B, slabs, M, N, Kd, M, N, N, trans_a=True, split_k=split, slab_stride=M * N, tile=tile, precision=prec)
    assert torch.isfinite(slabs).all()
    ref = A.t().double() @ B.double()
    assert rel_err(slabs.sum(0).double(), ref) < {"fp32": 1e-5, "bf16x3": 3e-5, "bf16": 2e-2}[prec]


def test_gemm_epilogues():
    M, N, Kd = 128, 128, 64
    A, B = _mk(M, Kd, seed=5), _mk(N, Kd, seed=6)
    bias, R = _mk(N, seed=7), _mk(M, N, seed=8)
    acc = A @ B.t()
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_BIAS, bias=bias, alpha=0.5, scale_cols=64)
    ref = acc + bias
    ref[:, :64] *= 0.5
    assert rel_err(C, ref) < 1e-5
    # dropout epilogues against the kernel's own mask
    p, seed = 0.5, 1234
    mask = K.dropout_mask(seed, M, N, p).float()
    assert 0.45 < mask.mean().item() < 0.55
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_BIAS_DROP_RESID, bias=bias, aux0=R,
           ld_aux=N, p_drop=p, seed=seed)
    assert rel_err(C, R + (acc + bias) * mask * 2) < 1e-5
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_BIAS_RELU_DROP, bias=bias, p_drop=p,
           seed=seed)
    H = torch.relu(acc + bias) * mask * 2
    assert rel_err(C, H) < 1e-5
    G = torch.empty(M, N, device=DEV)
    K.gemm(A, B, G, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_RELU_DROP_BWD, aux0=H, ld_aux=N, p_drop=p)
    assert rel_err(G, acc * (H > 0).float() * 2) < 1e-5
    C2 = R.clone()
    K.gemm(A, B, C2, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ACCUM, alpha=1.0)
    assert rel_err(C2, R + acc) < 1e-5
    P, Pd, dl = torch.rand(M, N, device=DEV), torch.rand(M, N, device=DEV), _mk(M, seed=9)
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ATTN_DS, aux0=P, aux1=Pd, rowvec=dl,
           ld_aux=N)
    assert rel_err(C, Pd * acc - P * dl[:, None]) < 1e-5


@pytest.mark.parametrize("Np,N", [(256, 200), (4864, 4776), (5376, 5300), (17408, 17000)])
def test_attn_softmax_masking_and_dropout(Np, N):
    S = _mk(Np, Np, seed=10) * 3
    P = torch.empty(Np, Np, device=DEV)
    K.attn_softmax_fwd(S, Np, P, P, Np, N, Np, N, Np, 0.0, 0)
    ref = torch.softmax(S[:N, :N], dim=1)
    assert rel_err(P[:N, :N], ref) < 1e-5
    assert P[:, N:].abs().max().item() == 0 and P[N:].abs().max().item() == 0
    Pd = torch.empty_like(P)
    K.attn_softmax_fwd(S, Np, P, Pd, Np, N, Np, N, Np, 0.5, 77)
    mask = K.dropout_mask(77, Np, Np, 0.5).float()
    assert rel_err(Pd[:N, :N], ref * mask[:N, :N] * 2) < 1e-5


def _unpack_bits(kb, cols):
    w = kb.to(torch.int64) & 0xFFFFFFFF
    bits = (w[:, :, None] >> torch.arange(32, device=kb.device)) & 1
    return bits.reshape(kb.shape[0], -1)[:, :cols]


@pytest.mark.parametrize("Np,N", [(1280, 1100), (256, 256), (2048, 1999), (4864, 4776), (9216, 9000)])
def test_attn_softmax_keep_bits(Np, N):
    """keep bits == the dropout mask on the valid block, 0 on padded rows/columns (n_pad not a
    multiple of the 1024-column trip included)."""
    S = _mk(Np, Np, seed=21)
    P, Pd = torch.empty(Np, Np, device=DEV), torch.empty(Np, Np, device=DEV)
    kb = torch.full((Np, Np // 32), -1, device=DEV, dtype=torch.int32)
    K.attn_softmax_fwd(S, Np, P, Pd, Np, N, Np, N, Np, 0.5, 99, keep=kb)
    bits = _unpack_bits(kb, Np)
    mask = K.dropout_mask(99, Np, Np, 0.5).to(torch.int64)
    assert torch.equal(bits[:N, :N], mask[:N, :N])
    assert bits[:, N:].sum().item() == 0 and bits[N:].sum().item() == 0
    assert torch.equal((Pd[:N, :N] != 0), (bits[:N, :N] == 1) & (P[:N, :N] != 0))


@pytest.mark.parametrize("prec", ["fp32", "bf16x3"])
def test_attn_ds_epilogue_with_keep_bits(prec):
    M = N = 256
    Kd = 64
    A, B = _mk(M, Kd, seed=31), _mk(N, Kd, seed=32)
    acc = A @ B.t()
    S = _mk(M, N, seed=33)
    P, Pd = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    kb = torch.empty(M, N // 32, device=DEV, dtype=torch.int32)
    K.attn_softmax_fwd(S, N, P, Pd, N, 230, M, 230, N, 0.5, 5, keep=kb)
    dl = _mk(M, seed=34)
    C1, C2 = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    K.gemm(A, B, C1, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ATTN_DS, aux0=P, aux1=Pd, rowvec=dl,
           ld_aux=N, precision=prec)
    K.gemm(A, B, C2, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ATTN_DS, aux0=P, keep=kb, p_drop=0.5,
           rowvec=dl, ld_aux=N, precision=prec)
    keep = _unpack_bits(kb, N).float()
    ref = P * (keep * acc * 2 - dl[:, None])
    assert rel_err(C2, ref) < (1e-5 if prec == "fp32" else 3e-5)
    assert rel_err(C2, C1) < 1e-5


@pytest.mark.parametrize("Np,N,p", [(1280, 1100, 0.5), (256, 230, 0.3), (9216, 9000, 0.5), (512, 500, 0.0)])
def test_attn_softmax_signed_image(Np, N, p):
    """P=None: one image, P/(1-p) where kept and -P where dropped (the sign bit is the keep bit,
    -0.0 for a dropped exact zero); bitwise equal to the two-buffer outputs elsewhere."""
    S = _mk(Np, Np, seed=23)
    P, Pd = torch.empty(Np, Np, device=DEV), torch.empty(Np, Np, device=DEV)
    K.attn_softmax_fwd(S, Np, P, Pd if p > 0 else P, Np, N, Np, N, Np, p, 77)
    X = torch.full((Np, Np), float("nan"), device=DEV)
    K.attn_softmax_fwd(S, Np, None if p > 0 else X, X, Np, N, Np, N, Np, p, 77)
    if p == 0:
        assert torch.equal(X, P)
        return
    mask = K.dropout_mask(77, Np, Np, p).bool()
    sign = torch.signbit(X)
    assert torch.equal(sign[:N, :N], ~mask[:N, :N])
    assert torch.equal(X[mask], Pd[mask])
    assert torch.equal(-X[~mask], P[~mask])
    assert X[N:].abs().max().item() == 0 and X[:, N:].abs().max().item() == 0


@pytest.mark.parametrize("prec", ["fp32", "bf16x3"])
@pytest.mark.parametrize("tile", [0, 256])
def test_clamp_a_and_signed_ds_epilogue(prec, tile):
    """The P.V / dP^T.dO products over the signed image (clamp_a) equal the products over Pd, and
    the ATTN_DS_SIGNED epilogue equals P * (keep * acc / (1-p) - delta)."""
    if prec == "fp32" and tile == 256:
        pytest.skip("256 tile is a bf16 mode")
    Np, N, dp, p = 512, 470, 128, 0.3
    S = _mk(Np, Np, seed=41)
    P, Pd, X = (torch.empty(Np, Np, device=DEV) for _ in range(3))
    K.attn_softmax_fwd(S, Np, P, Pd, Np, N, Np, N, Np, p, 9)
    K.attn_softmax_fwd(S, Np, None, X, Np, N, Np, N, Np, p, 9)
    V = _mk(Np, dp, seed=42)
    for ta in (False, True):
        O1, O2 = torch.empty(Np, dp, device=DEV), torch.empty(Np, dp, device=DEV)
        K.gemm(Pd, V, O1, Np, dp, Np, Np, dp, dp, trans_a=ta, precision=prec, tile=tile)
        K.gemm(X, V, O2, Np, dp, Np, Np, dp, dp, trans_a=ta, precision=prec, tile=tile, clamp_a=True)
        assert torch.equal(O1, O2)
        S3 = torch.empty(2, Np, dp, device=DEV)
        K.gemm(X, V, S3, Np, dp, Np, Np, dp, dp, trans_a=ta, precision=prec, tile=tile, clamp_a=True, split_k=2,
               slab_stride=Np * dp)
        assert rel_err(S3.sum(0), O1) < 1e-6
    dO = _mk(Np, dp, seed=43)
    acc = dO @ V.t()
    dl = _mk(Np, seed=44)
    C = torch.empty(Np, Np, device=DEV)
    K.gemm(dO, V, C, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_ATTN_DS_SIGNED, aux0=X, p_drop=p,
           rowvec=dl, ld_aux=Np, precision=prec, tile=tile)
    keep = K.dropout_mask(9, Np, Np, p).float()
    ref = P * (keep * acc / (1 - p) - dl[:, None])
    assert rel_err(C, ref) < (1e-5 if prec == "fp32" else 3e-5)
    with pytest.raises(_lib.U2GNNNativeError):   # clamp_a only with STORE and B not transposed
        K.gemm(dO, V, C, Np, Np, dp, dp, dp, Np, trans_b=True, precision=prec, clamp_a=True)
    with pytest.raises(_lib.U2GNNNativeError):   # the signed dS epilogue writes C only (no x2 copy)
        K.gemm(dO, V, C, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_ATTN_DS_SIGNED, aux0=X, p_drop=p,
               rowvec=dl, ld_aux=Np, precision=prec, tile=tile,
               Cx2=torch.empty(Np, 2 * Np, device=DEV, dtype=torch.bfloat16), ldcx2=2 * Np)


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
@pytest.mark.parametrize("p", [0.5, 0.0])
def test_signed_ds_lds_epilogue_128(prec, p):
    """The C4 dS kernel: ATTN_DS_SIGNED on 128x128 blocks with a 32-deep K step stages its result through LDS
    (gemm.hip ds_lds_store: row-contiguous image loads and dS stores).  Its per-element arithmetic is the
    MFMA-layout epilogue's, so the dS it writes is bit-identical to the 64x64 and 256x128 tiles' (same k-ordered
    sums) -- and within fp32 rounding of P * (keep * dO V^T / (1-p) - delta) in float64."""
    Np, N, dp = 512, 470, 384
    S = _mk(Np, Np, seed=61)
    P, Pd, X = (torch.empty(Np, Np, device=DEV) for _ in range(3))
    K.attn_softmax_fwd(S, Np, P, Pd if p > 0 else P, Np, N, Np, N, Np, p, 19)
    K.attn_softmax_fwd(S, Np, None if p > 0 else X, X, Np, N, Np, N, Np, p, 19)
    dO, V, dl = _mk(Np, dp, seed=62), _mk(Np, dp, seed=63), _mk(Np, seed=64)
    out = {}
    for tile in (128, 64, 256):
        C = torch.full((Np, Np), float("nan"), device=DEV)
        K.gemm(dO, V, C, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_ATTN_DS_SIGNED, aux0=X, p_drop=p,
               rowvec=dl, ld_aux=Np, precision=prec, tile=tile)
        out[tile] = C
    assert torch.isfinite(out[128]).all()
    assert torch.equal(out[128], out[64])
    assert torch.equal(out[128], out[256])
    keep = K.dropout_mask(19, Np, Np, p).double() if p > 0 else torch.ones(Np, Np, device=DEV, dtype=torch.float64)
    acc = dO.double() @ V.double().t()
    ref = P.double() * (keep * acc / (1 - p) - dl.double()[:, None])
    assert rel_err(out[128].double(), ref) < (3e-5 if prec == "bf16x3" else 2e-2)


@pytest.mark.parametrize("dp", [384, 640])   # 6 partials, and 10 (> the 8 held in registers)
@pytest.mark.parametrize("prec", ["fp32", "bf16x3", "bf16"])
@pytest.mark.parametrize("tile", [0, 64, 128])
def test_store_rowdot_partials_feed_signed_ds(prec, tile, dp):
    """ABI v8: the dO GEMM's STORE_ROWDOT epilogue stores C exactly as STORE and writes the row partials
    sum_{n in 64-column group q} C[m,n] * O[m,n]; ATTN_DS_SIGNED with those partials (rowvec_parts)
    equals the same epilogue fed delta = their sum in group order, and the rowdot delta to fp32 rounding."""
    Np, N, p = 512, 470, 0.3
    dA, Wo, O = _mk(Np, dp, seed=51), _mk(dp, dp, seed=52) * 0.05, _mk(Np, dp, seed=53)
    C0, C1 = torch.empty(Np, dp, device=DEV), torch.empty(Np, dp, device=DEV)
    parts = torch.full((dp // 64, Np + 64), float("nan"), device=DEV)[:, :Np + 16]   # ld_rowpart > M
    K.gemm(dA, Wo, C0, Np, dp, dp, dp, dp, dp, precision=prec, tile=tile)
    K.gemm(dA, Wo, C1, Np, dp, dp, dp, dp, dp, precision=prec, tile=tile, epilogue=_lib.EPI_STORE_ROWDOT, aux0=O,
           ld_aux=dp, rowpart=parts)
    assert torch.equal(C0, C1)
    ref = (C0.double() * O.double()).view(Np, dp // 64, 64).sum(2).t()
    assert torch.isfinite(parts[:, :Np]).all()
    assert rel_err(parts[:, :Np].double(), ref) < 1e-5
    delta_seq = torch.zeros(Np, device=DEV)
    for q in range(dp // 64):   # the dS epilogue's order
        delta_seq = delta_seq + parts[q, :Np]
    delta_rd = torch.empty(Np, device=DEV)
    K.rowdot(C1, dp, O, dp, delta_rd, Np, dp)
    assert rel_err(delta_seq, delta_rd) < 1e-5
    S = _mk(Np, Np, seed=54)
    X = torch.empty(Np, Np, device=DEV)
    K.attn_softmax_fwd(S, Np, None, X, Np, N, Np, N, Np, p, 9)
    V = _mk(Np, dp, seed=55)
    dS1, dS2 = torch.empty(Np, Np, device=DEV), torch.empty(Np, Np, device=DEV)
    K.gemm(C1, V, dS1, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_ATTN_DS_SIGNED, aux0=X, p_drop=p,
           rowvec=parts[:, :Np], ld_aux=Np, precision=prec)
    K.gemm(C1, V, dS2, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_ATTN_DS_SIGNED, aux0=X, p_drop=p,
           rowvec=delta_seq, ld_aux=Np, precision=prec)
    assert torch.equal(dS1, dS2)
    with pytest.raises(_lib.U2GNNNativeError):   # partials only for the dS epilogue
        K.gemm(C1, V, dS1, Np, Np, dp, dp, dp, Np, trans_b=True, aux0=X, rowvec=parts[:, :Np], ld_aux=Np,
               precision=prec)
    with pytest.raises(_lib.U2GNNNativeError):   # no split-K with the row partials
        K.gemm(dA, Wo, C1, Np, dp, dp, dp, dp, dp, precision=prec, epilogue=_lib.EPI_STORE_ROWDOT, aux0=O,
               ld_aux=dp, rowpart=parts, split_k=2, slab_stride=Np * dp)


def test_dropout_mask_statistics():
    """The counter-based keep decision: rate 1-p, no correlation between neighbouring rows, columns
    or seeds (the masks of the attention dropout are 2-D slices of this stream)."""
    R = C = 2048
    for p in (0.1, 0.5, 0.9):
        m = K.dropout_mask(1234, R, C, p).float()
        assert abs(m.mean().item() - (1 - p)) < 0.003
    m = K.dropout_mask(1234, R, C, 0.5).float() - 0.5
    m2 = K.dropout_mask(1235, R, C, 0.5).float() - 0.5

    def corr(a, b):
        return ((a * b).mean() / (a.std() * b.std())).abs().item()
    assert corr(m[:, 1:], m[:, :-1]) < 0.01
    assert corr(m[1:], m[:-1]) < 0.01
    assert corr(m, m2) < 0.01
    assert m.mean(1).std().item() < 4 * 0.5 / C ** 0.5   # per-row rates: binomial spread


@pytest.mark.parametrize("d,dp", [(67, 128), (200, 256), (367, 384), (500, 512), (600, 640), (1000, 1024)])
@pytest.mark.parametrize("gb_offset", [0, 1])   # 16-byte aligned gamma / beta (float4 loads) or not
def test_layernorm_fwd_bwd(d, dp, gb_offset):
    """Per-lane widths 1, 2, 3, 4 and the 8-wide fallback of the LayerNorm kernels."""
    Np, N = 128, 100
    Z = _mk(Np, dp, seed=11)
    gam, bet = _mk(d + gb_offset, seed=12)[gb_offset:], _mk(d + gb_offset, seed=13)[gb_offset:]
    Y = torch.empty(Np, dp, device=DEV)
    mu, rs = torch.empty(Np, device=DEV), torch.empty(Np, device=DEV)
    K.layernorm_fwd(Z, dp, gam, bet, Y, dp, mu, rs, N, Np, d, dp)
    z = Z[:N, :d].clone().requires_grad_(True)
    g_, b_ = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(z, (d,), g_, b_, 1e-5)
    assert rel_err(Y[:N, :d], ref) < 1e-5
    assert Y[:, d:].abs().max().item() == 0 and Y[N:].abs().max().item() == 0
    dY = torch.zeros(Np, dp, device=DEV)
    dY[:N, :d] = _mk(N, d, seed=14)
    ref.backward(dY[:N, :d])
    dZ, dZd = torch.empty(Np, dp, device=DEV), torch.empty(Np, dp, device=DEV)
    K.layernorm_bwd(dY, dp, Z, dp, mu, rs, gam, dZ, dp, dZd, dp, 0.5, 99, N, Np, d, dp)
    dg, db, dbias = torch.empty(d, device=DEV), torch.empty(d, device=DEV), torch.empty(d, device=DEV)
    ws = torch.empty(K.colstat_ws_floats(N, dp), device=DEV)
    K.layernorm_bwd_params(dY, dp, Z, dp, mu, rs, dZd, dp, N, d, dp, ws, dg, db, dbias)
    assert rel_err(dZ[:N, :d], z.grad) < 1e-4
    mask = K.dropout_mask(99, Np, dp, 0.5).float()
    assert rel_err(dZd[:N, :d], z.grad * mask[:N, :d] * 2) < 1e-4
    assert rel_err(dg, g_.grad) < 1e-4 and rel_err(db, b_.grad) < 1e-4
    assert rel_err(dbias, (z.grad * mask[:N, :d] * 2).sum(0)) < 1e-4
    assert dZ[N:].abs().max().item() == 0 and dZ[:, d:].abs().max().item() == 0


@pytest.mark.parametrize("d,K_,p", [(19, 64, 0.0), (19, 1024, 0.5), (64, 64, 0.5), (4, 64, 0.0)])
@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
@pytest.mark.parametrize("gb_offset", [0, 1])   # 16-byte aligned gamma / beta (float4 loads) or not
def test_bias_drop_resid_layernorm_epilogue(d, K_, p, prec, gb_offset):
    """EPI_BIAS_DROP_RESID_LN (d <= 64, one 64-column tile per row): Z is bit-identical to the
    BIAS_DROP_RESID epilogue, Y / mean / rstd match layernorm_fwd on that Z (fp32, 1e-5), rows past
    ln_rows and columns past d are zero."""
    Np, N, dp = 320, 300, 64
    A = _mk(Np, K_, seed=41)
    W = _mk(dp, K_, seed=42) * 0.1
    bias = _mk(dp, seed=43)
    X = _mk(Np, dp, seed=44)
    gam, bet = _mk(d + gb_offset, seed=45)[gb_offset:], _mk(d + gb_offset, seed=46)[gb_offset:]
    Z_ref = torch.empty(Np, dp, device=DEV)
    K.gemm(A, W, Z_ref, Np, dp, K_, K_, K_, dp, trans_b=True, epilogue=_lib.EPI_BIAS_DROP_RESID, bias=bias, aux0=X,
           ld_aux=dp, p_drop=p, seed=5, precision=prec)
    Z = torch.full((Np, dp), float("nan"), device=DEV)
    Y = torch.full((Np, dp), float("nan"), device=DEV)
    mu, rs = torch.full((Np,), float("nan"), device=DEV), torch.full((Np,), float("nan"), device=DEV)
    K.gemm(A, W, Z, Np, dp, K_, K_, K_, dp, trans_b=True, epilogue=_lib.EPI_BIAS_DROP_RESID_LN, bias=bias, aux0=X,
           ld_aux=dp, p_drop=p, seed=5, precision=prec, ln=(gam, bet, Y, dp, mu, rs, d, N, 1e-5))
    assert torch.equal(Z, Z_ref)
    Y_ref = torch.empty(Np, dp, device=DEV)
    mu_ref, rs_ref = torch.empty(Np, device=DEV), torch.empty(Np, device=DEV)
    K.layernorm_fwd(Z_ref, dp, gam, bet, Y_ref, dp, mu_ref, rs_ref, N, Np, d, dp)
    assert rel_err(Y, Y_ref) < 1e-5
    assert rel_err(mu, mu_ref) < 1e-5 and rel_err(rs, rs_ref) < 1e-5
    assert Y[N:].abs().max().item() == 0 and (d == dp or Y[:, d:].abs().max().item() == 0)
    assert mu[N:].abs().max().item() == 0 and rs[N:].abs().max().item() == 0


def test_gather_pack_colsum():
    src = _mk(50, 7, seed=15)
    idx = torch.randint(0, 50, (30, 5), device=DEV)
    dst = torch.full((64, 64), 7.0, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.gather_rows(src, idx, 5, dst, 30, 64, 7, 64, err)
    assert torch.equal(dst[:30, :7], src[idx[:, 0]]) and dst[30:].abs().max() == 0 and dst[:, 7:].abs().max() == 0
    assert err.item() == 0
    # out-of-range entries (F.embedding raises IndexError): gather writes zeros, scatter adds nothing,
    # both flag err and touch no memory outside the buffers
    bad = idx.clone()
    bad[3, 0], bad[7, 0] = 50, -1
    K.gather_rows(src, bad, 5, dst, 30, 64, 7, 64, err)
    assert err.item() == 1 and dst[3].abs().max() == 0 and dst[7].abs().max() == 0
    assert torch.equal(dst[4, :7], src[bad[4, 0]])
    err.zero_()
    acc = torch.zeros(50, 7, device=DEV)
    K.scatter_add_rows(src[:30], bad, 5, acc, 30, 7, err)
    good = torch.ones(30, dtype=torch.bool, device=DEV)
    good[3] = good[7] = False
    ref = torch.zeros(50, 7, device=DEV).index_add_(0, bad[good, 0], src[:30][good])
    assert err.item() == 1 and (acc - ref).abs().max().item() < 1e-5
    W = _mk(3 * 7, 7, seed=16)
    Wp = torch.empty(3 * 64, 64, device=DEV)
    K.pack_padded(W, 7, 3 * 64, 64, (64, 7), (64, 7), Wp, 64)
    for q in range(3):
        assert torch.equal(Wp[q * 64:q * 64 + 7, :7], W[q * 7:(q + 1) * 7])
    Wm = torch.full_like(Wp, 3.0)
    bsrc = _mk(21, seed=23)
    bm = torch.full((3 * 64,), 5.0, device=DEV)
    K.pack_padded_multi([(W, 7, 3 * 64, 64, (64, 7), (64, 7), Wm, 64), (bsrc, 21, 1, 3 * 64, (1, 1), (64, 7), bm, 192)])
    assert torch.equal(Wm, Wp) and bm.view(3, 64)[:, 7:].abs().max() == 0
    assert torch.equal(bm.view(3, 64)[:, :7].reshape(-1), bsrc)
    X = _mk(300, 192, seed=17)
    out = torch.empty(3 * 7, device=DEV)
    ws = torch.empty(K.colstat_ws_floats(300, 192), device=DEV)   # >= ceil(300/16) * 192 (u2gnn_hip.h)
    K.colsum(X, 300, 192, 192, (64, 7), out, ws)
    ref = X.sum(0).view(3, 64)[:, :7].reshape(-1)
    assert rel_err(out, ref) < 1e-5


@pytest.mark.parametrize("N,Np,d,dp,p", [(470, 512, 367, 384, 0.5), (300, 320, 19, 64, 0.3), (200, 256, 65, 128, 0.0)])
def test_layernorm_bwd_delta_equals_rowdot(N, Np, d, dp, p):
    """LayerNorm1's backward with the attention delta (ABI v8): dZ / dZdrop bit-identical to
    layernorm_bwd, and delta = sum_c dZdrop * ((Z - X)(1-p) - b_o) equal to rowdot(dO, O) with
    dO = dZdrop W_o (fp32 products; 1e-5 of the row scale), 0 on padded rows."""
    seed = 321
    O = torch.zeros(Np, dp, device=DEV)
    O[:N, :d] = _mk(N, d, seed=71)
    X = torch.zeros(Np, dp, device=DEV)
    X[:N, :d] = _mk(N, d, seed=72)
    Wo = torch.zeros(dp, dp, device=DEV)
    Wo[:d, :d] = _mk(d, d, seed=73) / math.sqrt(d)
    bo = torch.zeros(dp, device=DEV)
    bo[:d] = _mk(d, seed=74) * 0.1
    Z = torch.empty(Np, dp, device=DEV)   # the executor's out-projection: Z = X + drop(O W_o^T + b_o)
    K.gemm(O, Wo, Z, Np, dp, dp, dp, dp, dp, trans_b=True, epilogue=_lib.EPI_BIAS_DROP_RESID, bias=bo, aux0=X,
           ld_aux=dp, p_drop=p, seed=seed)
    gam = _mk(d, seed=75)
    bet = _mk(d, seed=76)
    Y, mean, rstd = torch.empty(Np, dp, device=DEV), torch.empty(Np, device=DEV), torch.empty(Np, device=DEV)
    K.layernorm_fwd(Z, dp, gam, bet, Y, dp, mean, rstd, N, Np, d, dp)
    dY = torch.zeros(Np, dp, device=DEV)
    dY[:N, :d] = _mk(N, d, seed=77)
    dZ1, dA1, dZ2, dA2 = (torch.full((Np, dp), float("nan"), device=DEV) for _ in range(4))
    K.layernorm_bwd(dY, dp, Z, dp, mean, rstd, gam, dZ1, dp, dA1, dp, p, seed, N, Np, d, dp)
    delta = torch.full((Np,), float("nan"), device=DEV)
    K.layernorm_bwd_delta(dY, dp, Z, dp, mean, rstd, gam, dZ2, dp, dA2, dp, p, seed, N, Np, d, dp, X, dp, bo, delta)
    assert torch.equal(dZ1, dZ2) and torch.equal(dA1, dA2)
    dO = dA2.double() @ Wo.double()
    ref = (dO * O.double()).sum(1)
    scale = ((dO.abs() * O.double().abs()).sum(1)).max().item()
    assert (delta.double() - ref).abs().max().item() < 1e-5 * scale
    assert delta[N:].abs().max().item() == 0
    with pytest.raises(_lib.U2GNNNativeError):
        K.layernorm_bwd_delta(dY, dp, Z, dp, mean, rstd, gam, dZ2, dp, dA2, dp, p, seed, N, Np, d, dp, X[:, 1:], dp,
                              bo, delta)   # misaligned X


def test_pack_multi_c4_shapes_equal_single_jobs():
    """The batched pack (8 rows per block, 32-bit maps) writes exactly what one pack_padded launch per
    job writes: C4's in-projection (3 row blocks), FFN weights, a bias row with 3 column blocks, and a
    job whose padded row count is not a multiple of 8."""
    d, dp, ff = 367, 384, 1024
    shapes = [  # (real rows, real cols, rows_pad, cols_pad, rblk, cblk)
        (3 * d, d, 3 * dp, dp, (dp, d), (dp, d)),
        (ff, d, ff, dp, (ff, ff), (dp, d)),
        (d, ff, dp, ff, (dp, d), (ff, ff)),
        (1, 3 * d, 1, 3 * dp, (1, 1), (dp, d)),
        (3 * 5, 7, 3 * 7, 64, (7, 5), (64, 7)),
    ]
    jobs, singles = [], []
    for i, (r, c, rp, cp, rb, cb) in enumerate(shapes):
        src = _mk(r, c, seed=60 + i)
        a, b = torch.full((rp, cp), 9.0, device=DEV), torch.full((rp, cp), -9.0, device=DEV)
        jobs.append((src, c, rp, cp, rb, cb, a, cp))
        K.pack_padded(src, c, rp, cp, rb, cb, b, cp)
        singles.append(b)
    K.pack_padded_multi(jobs)
    for j, b in zip(jobs, singles):
        assert torch.equal(j[6], b)
    Wp = singles[0]   # spot check of the block map against the real matrix
    W = jobs[0][0]
    for q in range(3):
        assert torch.equal(Wp[q * dp:q * dp + d, :d], W[q * d:(q + 1) * d])
        assert Wp[q * dp + d:(q + 1) * dp].abs().max().item() == 0 and Wp[:, d:].abs().max().item() == 0


@pytest.mark.parametrize("rows", [1, 255, 2000, 2560, 2561, 4864, 8192, 8209, 20011, 82110])
def test_column_reductions_token_sized(rows):
    """colsum / LN parameter sums against torch float64, from one row to neighbour-mode row counts
    (those fold several 16-row groups into one chunk: at most 512 chunks, the ragged last one
    included)."""
    d, dp = 367, 384
    X = torch.zeros(rows, dp, device=DEV)
    X[:, :d] = _mk(rows, d, seed=31)
    out = torch.empty(d, device=DEV)
    ws = torch.full((K.colstat_ws_floats(rows, dp),), float("nan"), device=DEV)
    K.colsum(X, rows, dp, dp, (dp, d), out, ws)
    ref = X[:, :d].double().sum(0)
    assert (out.double() - ref).abs().max().item() < 1e-5 * rows ** 0.5 * 4
    Z = torch.zeros(rows, dp, device=DEV)
    Z[:, :d] = _mk(rows, d, seed=32)
    dY = torch.zeros(rows, dp, device=DEV)
    dY[:, :d] = _mk(rows, d, seed=33)
    dZd = torch.zeros(rows, dp, device=DEV)
    dZd[:, :d] = _mk(rows, d, seed=34)
    mu = Z[:, :d].mean(1)
    rs = torch.rsqrt(Z[:, :d].var(1, unbiased=False) + 1e-5)
    dg, db, dbias = (torch.empty(d, device=DEV) for _ in range(3))
    ws.fill_(float("nan"))
    K.layernorm_bwd_params(dY, dp, Z, dp, mu, rs, dZd, dp, rows, d, dp, ws, dg, db, dbias)
    xh = ((Z[:, :d] - mu[:, None]) * rs[:, None]).double()
    tol = 1e-5 * rows ** 0.5 * 4
    assert (dg.double() - (dY[:, :d].double() * xh).sum(0)).abs().max().item() < tol
    assert (db.double() - dY[:, :d].double().sum(0)).abs().max().item() < tol
    assert (dbias.double() - dZd[:, :d].double().sum(0)).abs().max().item() < tol


@pytest.mark.parametrize("d,d_pad,ld_src,n_src,n_rows,n_pad,ld_dst", [
    (367, 384, 367, 500, 4099, 4352, 384),  # X_concat at C4 width: 4-byte-aligned rows (multi kernel, wide)
    (367, 384, 367, 500, 4099, 4102, 384),  # rows_pad not a multiple of the 32 rows of one XCD block round
    (384, 384, 384, 300, 1000, 1024, 384),  # padded [Np, dp] re-gather: 16-byte rows (mode 1)
    (7, 64, 7, 50, 30, 64, 64),             # MUTAG width (multi kernel, wide)
    (5, 66, 5, 40, 33, 40, 68),             # d_pad % 4 != 0 (multi kernel, dword stores)
    (5, 66, 5, 40, 33, 40, 66),             # dst rows not 16-byte aligned (mode 2)
    (600, 640, 600, 40, 70, 80, 640),       # 512 < d_pad <= 1024 (mode 2)
    (6, 64, 8, 40, 33, 64, 64),             # aligned source, d % 4 != 0 (mode 1 tail)
    (1100, 1152, 1100, 20, 17, 64, 1152),   # d_pad > 1024 (mode 0 loop)
])
def test_gather_rows_modes(d, d_pad, ld_src, n_src, n_rows, n_pad, ld_dst):
    """a2 gather (pytorch_U2GNN_Sup.py:32): bit-exact copy of the indexed rows, zero padding, and
    out-of-range indices reported through err with a zero row; columns past d_pad untouched."""
    g = torch.Generator(device="cpu").manual_seed(d + n_rows)
    src_full = torch.randn(n_src, ld_src, generator=g).to(DEV)
    idx = torch.randint(0, n_src, (n_rows, 2), generator=g)
    idx[n_rows // 2, 0] = n_src          # out of range -> zero row, err = 1
    idx = idx.to(DEV)
    dst_full = torch.full((n_pad, ld_dst), 7.0, device=DEV)
    dst = dst_full[:, :d_pad]
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.gather_rows(src_full, idx, 2, dst, n_rows, n_pad, d, d_pad, err)
    ref = torch.full((n_pad, ld_dst), 7.0, device=DEV)
    ref[:, :d_pad] = 0
    ok = idx[:, 0] < n_src
    ref[:n_rows, :d][ok] = src_full[idx[ok, 0], :d]
    assert torch.equal(dst_full, ref)
    assert err.item() == 1


def test_pool_head_ce():
    Np, d, dp, B, C = 128, 10, 64, 4, 3
    X = _mk(Np, dp, seed=18)
    off = torch.tensor([0, 5, 9, 70, 128], device=DEV)
    col = torch.arange(128, device=DEV)
    vals = torch.ones(128, device=DEV)
    G = torch.zeros(B, dp, device=DEV)
    K.pool_fwd(X, dp, off, col, vals, G, dp, B, d, 0.0, 0)
    ref = torch.stack([X[off[b]:off[b + 1], :d].sum(0) for b in range(B)])
    assert rel_err(G[:, :d], ref) < 1e-5
    W, bias = _mk(C, d, seed=19), _mk(C, seed=20)
    sc = torch.empty(B, C, device=DEV)
    K.head_fwd(G, dp, W, bias, sc, B, C, d, False)
    assert rel_err(sc, ref @ W.t() + bias) < 1e-5
    labels = torch.tensor([0, 2, 1, 2], device=DEV)
    loss, ds = torch.empty(1, device=DEV), torch.empty(B, C, device=DEV)
    K.smoothed_ce(sc, labels, B, C, 0.1, loss, ds)
    s = sc.clone().requires_grad_(True)
    t = torch.full((B, C), 0.05, device=DEV)
    t.scatter_(1, labels[:, None], 0.9)
    lref = torch.mean(torch.sum(-t * torch.log_softmax(s, 1), 1))
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-5 and rel_err(ds, s.grad) < 1e-5


@pytest.mark.parametrize("B,N,Np,d,dp,p", [(4, 100, 128, 10, 64, 0.3), (64, 4776, 4864, 367, 384, 0.5),
                                            (3, 256, 256, 65, 128, 0.0)])
def test_pool_bwd_rows_equals_accumulating_pool_bwd(B, N, Np, d, dp, p):
    """ABI v8 block-row pool backward (plain stores, no zero fill) == the accumulating kernel into a
    zero-filled buffer: graph rows, padding columns d..dp and padding rows N..Np; and head_bwd's
    16-deep load batches leave its dW / db / dG equal to a float64 reference."""
    g = torch.Generator().manual_seed(5)
    cuts = torch.sort(torch.randperm(N - 1, generator=g)[:B - 1] + 1).values
    off = torch.cat([torch.tensor([0]), cuts, torch.tensor([N])]).to(DEV)
    col = torch.arange(N, device=DEV)
    vals = torch.rand(N, generator=g).to(DEV) + 0.5
    dG = _mk(B, dp, seed=81)
    ref = torch.zeros(Np, dp, device=DEV)
    K.pool_bwd(dG, dp, off, col, vals, ref, dp, B, d, p, 17)
    out = torch.full((Np, dp), float("nan"), device=DEV)
    K.pool_bwd_rows(dG, dp, off, col, vals, out, dp, B, d, dp, N, Np, p, 17)
    assert torch.equal(out, ref)
    C = 3
    G, W, dS = _mk(B, dp, seed=82), _mk(C, d, seed=83), _mk(B, C, seed=84)
    dGo, dW, db = torch.empty(B, dp, device=DEV), torch.empty(C, d, device=DEV), torch.empty(C, device=DEV)
    K.head_bwd(dS, G, dp, W, dGo, dp, dW, db, B, C, d)
    assert rel_err(dW.double(), dS.double().t() @ G[:, :d].double()) < 1e-5
    assert rel_err(db.double(), dS.double().sum(0)) < 1e-5
    assert rel_err(dGo[:, :d].double(), dS.double() @ W.double()) < 1e-5


def test_adam_matches_torch():
    n = 1000
    p0 = _mk(n, seed=21)
    g = _mk(n, seed=22) * 3
    p1 = p0.clone()
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    ws, sq = torch.empty(1024, device=DEV), torch.empty(1, device=DEV)
    tp = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([tp], lr=0.01)
    for step in range(1, 4):
        K.sqnorm(g, n, ws, sq)
        K.adam(p1, g, m, v, n, sq, 0.5, 0.9, 0.999, 1e-8, 0.01 / (1 - 0.9 ** step), math.sqrt(1 - 0.999 ** step))
        tp.grad = g.clone()
        torch.nn.utils.clip_grad_norm_([tp], 0.5)
        opt.step()
    assert abs(sq.item() - (g.double() ** 2).sum().item()) / sq.item() < 1e-5
    assert rel_err(p1, tp.detach()) < 1e-5


# ---- ABI v11: batched reductions and grouped weight-gradient GEMMs (bit-identical to single calls) ----
@pytest.mark.parametrize("rows", [300, 1920, 20000])   # small forms, long forms, folded long forms
def test_reduce_batch_equals_single_jobs(rows):
    d, dp, ff, ffp = 19, 64, 100, 128
    g = torch.Generator(device=DEV).manual_seed(11)
    rn = lambda *s: torch.randn(*s, device=DEV, generator=g)   # noqa: E731
    dY, Z, dZd = rn(rows, dp), rn(rows, dp), rn(rows, dp)
    mean, rstd = rn(rows), rn(rows).abs() + 0.5
    X = rn(rows, ffp)
    slabs = rn(6, ffp, dp)
    ref = {k: torch.full((n,), float("nan"), device=DEV) for k, n in
           (("gam", d), ("bet", d), ("bia", d), ("gam2", d), ("bet2", d), ("cs", ff))}
    ref["w"] = torch.full((ff, d), float("nan"), device=DEV)
    ref["acc"] = rn(ffp, dp)
    out = {k: v.clone() for k, v in ref.items()}
    ws = torch.empty(K.colstat_ws_floats(rows, ffp), device=DEV)
    K.layernorm_bwd_params(dY, dp, Z, dp, mean, rstd, dZd, dp, rows, d, dp, ws, ref["gam"], ref["bet"], ref["bia"])
    K.layernorm_bwd_params(dY, dp, Z, dp, mean, rstd, None, dp, rows, d, dp, ws, ref["gam2"], ref["bet2"], None)
    K.colsum(X, rows, ffp, ffp, (ffp, ff), ref["cs"], ws)
    K.slab_reduce(slabs, 6, ffp * dp, ffp, dp, dp, (ffp, ff), (dp, d), ref["w"], d, alpha=0.5)
    K.slab_reduce(slabs, 6, ffp * dp, ffp, dp, dp, (ffp, ffp), (dp, dp), ref["acc"], dp, accumulate=True)
    R = _lib
    jobs = [
        dict(kind=R.RJOB_LNPARAMS, src=dY, ld_src=dp, Z=Z, ldz=dp, mean=mean, rstd=rstd, dZdrop=dZd, lddrop=dp,
             rows=rows, d=d, cols=dp, dst=out["gam"], dbeta=out["bet"], dbias=out["bia"]),
        dict(kind=R.RJOB_SLAB, src=slabs, n_slab=6, slab_stride=ffp * dp, rows=ffp, cols=dp, ld_src=dp,
             rblk_pad=ffp, rblk_real=ff, cblk_pad=dp, cblk_real=d, dst=out["w"], ld_dst=d, alpha=0.5),
        dict(kind=R.RJOB_COLSUM, src=X, rows=rows, cols=ffp, ld_src=ffp, cblk_pad=ffp, cblk_real=ff, dst=out["cs"]),
        dict(kind=R.RJOB_LNPARAMS, src=dY, ld_src=dp, Z=Z, ldz=dp, mean=mean, rstd=rstd, rows=rows, d=d, cols=dp,
             dst=out["gam2"], dbeta=out["bet2"]),
        dict(kind=R.RJOB_SLAB, src=slabs, n_slab=6, slab_stride=ffp * dp, rows=ffp, cols=dp, ld_src=dp,
             rblk_pad=ffp, rblk_real=ffp, cblk_pad=dp, cblk_real=dp, dst=out["acc"], ld_dst=dp, alpha=1.0,
             accumulate=1),
    ]
    K.reduce_batch(jobs)
    torch.cuda.synchronize()
    for k in ref:
        assert torch.isfinite(out[k]).all(), k
        assert torch.equal(out[k], ref[k]), k


def test_reduce_batch_rejects_bad_jobs():
    x = torch.zeros(64, 64, device=DEV)
    with pytest.raises(_lib.U2GNNNativeError):
        K.reduce_batch([dict(kind=7, src=x, dst=x)])
    with pytest.raises(_lib.U2GNNNativeError):   # LN job without mean / rstd
        K.reduce_batch([dict(kind=_lib.RJOB_LNPARAMS, src=x, ld_src=64, Z=x, ldz=64, rows=64, d=4, cols=64, dst=x,
                             dbeta=x)])


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
@pytest.mark.parametrize("tile", [64, 129])
def test_gemm_group_equals_single_calls(prec, tile):
    # the weight-gradient shapes of a d <= 64 layer (dY^T X over Np rows) with split-K slabs
    Np, shapes = 2048, [(64, 1024, 16), (1024, 64, 16), (64, 64, 16), (192, 64, 8)]
    if tile == 129:
        shapes = [(128, 1024, 4), (1024, 128, 4), (384, 128, 8)]
    calls, outs, refs = [], [], []
    for i, (M, N, split) in enumerate(shapes):
        A, B = _mk(Np, M, seed=10 + i), _mk(Np, N, seed=20 + i)
        o, r = torch.full((split, M, N), float("nan"), device=DEV), torch.full((split, M, N), float("nan"), device=DEV)
        kw = dict(A=A, B=B, C=o, M=M, N=N, K=Np, lda=M, ldb=N, ldc=N, trans_a=True, split_k=split,
                  slab_stride=M * N, precision=prec, tile=tile)
        K.gemm(**dict(kw, C=r))
        calls.append(kw)
        outs.append(o)
        refs.append(r)
    K.gemm_group(calls)
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.equal(o, r)


def test_gemm_group_mixed_configurations_fall_back():
    A, B = _mk(512, 128, seed=1), _mk(512, 64, seed=2)
    c1, c2 = torch.empty(128, 64, device=DEV), torch.empty(128, 64, device=DEV)
    r1, r2 = torch.empty_like(c1), torch.empty_like(c2)
    k1 = dict(A=A, B=B, C=c1, M=128, N=64, K=512, lda=128, ldb=64, ldc=64, trans_a=True, precision="bf16x3", tile=64)
    k2 = dict(A=A, B=B, C=c2, M=128, N=64, K=512, lda=128, ldb=64, ldc=64, trans_a=True, precision="fp32", tile=64)
    K.gemm(**dict(k1, C=r1))
    K.gemm(**dict(k2, C=r2))
    K.gemm_group([k1, k2])
    torch.cuda.synchronize()
    assert torch.equal(c1, r1) and torch.equal(c2, r2)


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
@pytest.mark.parametrize("tile,Np,dp,split", [(64, 512, 64, 7), (256, 1024, 128, 4)])
def test_gemm_group_attention_layouts(prec, tile, Np, dp, split):
    # the attention backward's products in one launch: dV = clamp0(Pd)^T dO, dQ = dS K, dK = dS^T Q
    Pd = _mk(Np, Np, seed=3)            # signed image: negative entries are read as 0 (clamp_a)
    dS, dO, QKV = _mk(Np, Np, seed=4), _mk(Np, dp, seed=5), _mk(Np, 3 * dp, seed=6)
    base = dict(M=Np, N=dp, K=Np, ldc=dp, split_k=split, slab_stride=Np * dp, precision=prec, tile=tile)
    jobs = [dict(base, A=Pd, B=dO, lda=Np, ldb=dp, trans_a=True, clamp_a=True),
            dict(base, A=dS, B=QKV[:, dp:], lda=Np, ldb=3 * dp, alpha=0.25),
            dict(base, A=dS, B=QKV, lda=Np, ldb=3 * dp, trans_a=True)]
    outs, refs = [], []
    for kw in jobs:
        r = torch.full((split, Np, dp), float("nan"), device=DEV)
        K.gemm(**dict(kw, C=r))
        kw["C"] = torch.full_like(r, float("nan"))
        outs.append(kw["C"])
        refs.append(r)
    K.gemm_group(jobs)
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.isfinite(o).all()
        assert torch.equal(o, r)


# ---- ABI v11: UnSup head glue, each against the launches it replaces ----
@pytest.mark.parametrize("L,p", [(1, 0.5), (3, 0.3), (2, 0.0)])
def test_concat_and_split_dropout_equal_separate_launches(L, p):
    N, Np, d, dp, seed = 1914, 2048, 4, 64, 1234567
    outs = [_mk(Np, dp, seed=40 + l) for l in range(L)]
    D = d * L
    OV = torch.empty(N, D, device=DEV)
    for l in range(L):
        K.slab_reduce(outs[l], 1, 0, N, dp, dp, (N, N), (dp, d), OV[:, l * d:], D)
    ref = torch.empty_like(OV)
    K.dropout(OV, D, ref, D, N, D, p, seed) if p > 0 else ref.copy_(OV)
    got = torch.full_like(OV, float("nan"))
    K.concat_dropout(outs, dp, N, d, got, D, p, seed)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    dY = _mk(N, D, seed=50)
    dd = dY.clone()
    if p > 0:
        K.dropout(dd, D, dd, D, N, D, p, seed)
    refs = []
    for l in range(L):
        r = torch.empty(Np, dp, device=DEV)
        K.pack_padded(dd[:, l * d:], D, Np, dp, (Np, N), (dp, d), r, dp)
        refs.append(r)
    gots = [torch.full((Np, dp), float("nan"), device=DEV) for _ in range(L)]
    K.split_dropout_bwd(dY, D, N, Np, d, dp, p, seed, gots)
    torch.cuda.synchronize()
    for g_, r in zip(gots, refs):
        assert torch.equal(g_, r)


@pytest.mark.parametrize("n", [1, 1000, 1914, 70001])
def test_sum_all_and_index_zero_rows2(n):
    x = _mk(n, seed=60)
    out = torch.full((1,), float("nan"), device=DEV)
    K.sum_all(x, n, out)
    torch.cuda.synchronize()
    assert abs(out.item() - x.double().sum().item()) <= 1e-5 * max(1.0, x.abs().sum().item())
    W = _mk(500, 4, seed=61)
    a = torch.tensor([3, 7, 499], device=DEV)
    b = torch.tensor([7, 0], device=DEV)
    ref = W.clone()
    ref[a] = 0
    ref[b] = 0
    K.index_zero_rows2(a, b, W)
    torch.cuda.synchronize()
    assert torch.equal(W, ref)


@pytest.mark.parametrize("d,p,rows,Np,n_slab", [(4, 0.5, 1914, 2048, 8), (19, 0.0, 1914, 2048, 8),
                                                 (64, 0.3, 1914, 2048, 8), (136, 0.5, 80, 128, 8),
                                                 (100, 0.0, 300, 384, 5), (256, 0.3, 250, 256, 3)])
def test_slab_bias_drop_resid_ln_against_fp64(d, p, rows, Np, n_slab):
    """d <= 64 (one column per lane) and the round-5 widths up to 256 (C2's IMDBBINARY: d = 136, dp = 192)."""
    seed, eps = 987654321, 1e-5
    dp = -(-d // 64) * 64
    slabs = _mk(n_slab, Np, dp, seed=70)
    bias = torch.zeros(dp, device=DEV)
    bias[:d] = _mk(d, seed=71)
    resid = _mk(Np, dp, seed=72)
    gamma, beta = _mk(d, seed=73), _mk(d, seed=74)
    Z, Y = torch.full((Np, dp), float("nan"), device=DEV), torch.full((Np, dp), float("nan"), device=DEV)
    mean, rstd = torch.full((Np,), float("nan"), device=DEV), torch.full((Np,), float("nan"), device=DEV)
    K.slab_bias_drop_resid_ln(slabs, n_slab, Np * dp, bias, resid, p, seed, Z, gamma, beta, Y, mean, rstd, d, rows, Np,
                              eps)
    torch.cuda.synchronize()
    x = slabs.double().sum(0) + bias.double()
    if p > 0:
        keep = K.dropout_mask(seed, Np, dp, p).bool()
        x = torch.where(keep, x / (1 - p), torch.zeros_like(x))
    zr = resid.double() + x
    assert ((Z.double()[:rows] - zr[:rows]).abs().max() / zr[:rows].abs().max()).item() < 1e-6
    assert torch.equal(Z[rows:], torch.zeros_like(Z[rows:]))   # padding rows: 0 (round 5)
    zd = Z.double()[:, :d]
    mu = zd.mean(1, keepdim=True)
    rs = 1.0 / torch.sqrt(((zd - mu) ** 2).mean(1, keepdim=True) + eps)
    yr = torch.zeros(Np, dp, dtype=torch.float64, device=DEV)
    yr[:rows, :d] = ((zd - mu) * rs * gamma.double() + beta.double())[:rows]
    assert (Y.double() - yr).abs().max().item() < 1e-4
    assert torch.equal(mean[rows:], torch.zeros_like(mean[rows:])) and torch.equal(rstd[rows:], torch.zeros_like(rstd[rows:]))
    assert (mean[:rows].double() - mu[:rows, 0]).abs().max().item() < 1e-5


@pytest.mark.parametrize("N,Np,d,dp,n_slab", [(1914, 2048, 4, 64, 14), (300, 384, 19, 64, 5), (1000, 1024, 367, 384, 3)])
def test_layernorm_bwd_delta_slabs_equals_reduce_then_ln(N, Np, d, dp, n_slab):
    p, seed = 0.5, 4242
    g = torch.Generator(device=DEV).manual_seed(5)
    rn = lambda *s: torch.randn(*s, device=DEV, generator=g)   # noqa: E731
    base, slabs, Z, X = rn(Np, dp), rn(n_slab, Np, dp), rn(Np, dp), rn(Np, dp)
    mean, rstd, gamma = rn(Np), rn(Np).abs() + 0.5, rn(d)
    bias = torch.zeros(dp, device=DEV)
    bias[:d] = rn(d)
    outs = []
    for fused in (False, True):
        dY = base.clone()
        dZ, dA, delta = torch.empty(Np, dp, device=DEV), torch.empty(Np, dp, device=DEV), torch.empty(Np, device=DEV)
        if fused:
            K.layernorm_bwd_delta_slabs(dY, dp, slabs, n_slab, Np * dp, Z, dp, mean, rstd, gamma, dZ, dp, dA, dp, p, seed,
                                        N, Np, d, dp, X, dp, bias, delta)
        else:
            K.slab_reduce(slabs, n_slab, Np * dp, Np, dp, dp, (Np, Np), (dp, dp), dY, dp, accumulate=True)
            K.layernorm_bwd_delta(dY, dp, Z, dp, mean, rstd, gamma, dZ, dp, dA, dp, p, seed, N, Np, d, dp, X, dp, bias,
                                  delta)
        outs.append((dY[:N], dZ, dA, delta))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [1001, 10 * 1024 * 1024 + 3])
def test_adam_sq_equals_sqnorm_then_adam(n):
    g = torch.Generator(device=DEV).manual_seed(9)
    grad = torch.randn(n, device=DEV, generator=g) * 0.1
    base = [torch.randn(n, device=DEV, generator=g) for _ in range(3)]
    base[2] = base[2].abs()
    out = []
    for fused in (False, True):
        p, m, v = (t.clone() for t in base)
        ws, sq = torch.zeros(1024, device=DEV), torch.full((1,), float("nan"), device=DEV)
        if fused:
            K.sqnorm_partials(grad, n, ws)
            K.adam_sq(p, grad, m, v, n, ws, sq, 0.5, 0.9, 0.999, 1e-8, 0.01, 0.3)
        else:
            K.sqnorm(grad, n, ws, sq)
            K.adam(p, grad, m, v, n, sq, 0.5, 0.9, 0.999, 1e-8, 0.01, 0.3)
        out.append((p, m, v, sq))
    torch.cuda.synchronize()
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("col0", [0, 128, 256])
def test_cx2_output_from_column(col0):
    """ABI v12 cx2_col0: the epilogue's x2 copy covers only columns >= col0 (the in-projection writes the x2
    copy of its V block only); those columns equal split_x2 of the fp32 result, the others stay untouched."""
    M, N, Kd = 256, 384, 64
    A, B = _mk(M, Kd, seed=3), _mk(N, Kd, seed=4)
    C = torch.empty(M, N, device=DEV)
    sentinel = torch.full((M, 2 * N), 7.0, device=DEV, dtype=torch.bfloat16)
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, precision="bf16x3", Cx2=sentinel, ldcx2=2 * N, cx2_col0=col0)
    ref = torch.empty(M, 2 * N, device=DEV, dtype=torch.bfloat16)
    K.split_x2(C, N, ref, 2 * N, M, N)
    torch.cuda.synchronize()
    assert torch.equal(sentinel[:, 2 * col0:], ref[:, 2 * col0:])
    assert bool((sentinel[:, :2 * col0] == 7.0).all())



def test_retired_gemm_modes_are_rejected():
    """ABI v13: the pre-split (x2) operands and the recomputed-P dS epilogue (ATTN_DS_RECOMP) that served
    them are gone; a call asking for either returns an error before any launch."""
    M = N = Kd = 128
    A, B, C = _mk(M, Kd, seed=5), _mk(N, Kd, seed=6), torch.empty(M, N, device=DEV)
    with pytest.raises(_lib.U2GNNNativeError):
        K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, precision="bf16x3", epilogue=_lib.EPI_ATTN_DS_RECOMP,
               aux0=C, rowvec=_mk(M, seed=7), ld_aux=N, p_drop=0.5)
    with pytest.raises(_lib.U2GNNNativeError):   # bf16 operands = the retired x2 form
        K.gemm(A.bfloat16(), B.bfloat16(), C, M, N, Kd, Kd, Kd, N, trans_b=True, precision="bf16x3")
    a = K._gemm_args(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, precision="bf16x3")
    a.a_x2 = a.b_x2 = 1
    assert K.hip_lib().u2gnn_gemm(ctypes.byref(a), None) == -1
    assert not hasattr(K.hip_lib(), "u2gnn_attn_softmax_x2_fwd")   # no longer exported
