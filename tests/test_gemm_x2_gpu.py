"""Pre-split (x2) attention path: split kernel, x2 GEMM (gemm_x2.hip) against the fp32-operand
BF16X3 GEMM (bit-identical on the same tile) and a float64 reference, softmax_x2 against the signed
softmax, and the recomputed-P dS epilogue against the signed-image dS epilogue."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import _lib as E  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402


def to_x2(X):
    R, C = X.shape
    out = torch.empty(R, 2 * C, device=X.device, dtype=torch.bfloat16)
    K.split_x2(X, X.stride(0), out, out.stride(0), R, C)
    return out


def from_x2(X2):
    R, C2 = X2.shape
    v = X2.view(R, C2 // 16, 2, 8).float()
    return (v[:, :, 0, :] + v[:, :, 1, :]).reshape(R, C2 // 2), v[:, :, 0, :].reshape(R, C2 // 2)


def test_split_x2_is_rne_hi_lo():
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(257, 96, device="cuda", generator=g) * torch.logspace(-3, 3, 96, device="cuda")
    X2 = to_x2(X)
    hi = X.to(torch.bfloat16)
    lo = (X - hi.float()).to(torch.bfloat16)
    v = X2.view(257, 12, 2, 8)
    assert torch.equal(v[:, :, 0, :].reshape(257, 96), hi)
    assert torch.equal(v[:, :, 1, :].reshape(257, 96), lo)
    rec, _ = from_x2(X2)
    assert ((rec - X).abs() <= X.abs() * 2.0 ** -16).all()


# (M, N, K, trans_a, trans_b, tile, split)
CASES = [
    (512, 384, 256, False, True, 256, 1),    # Q.K^T shape class (NT)
    (512, 384, 512, False, False, 256, 3),   # P.V (NN, split-K, ragged)
    (512, 384, 512, True, False, 256, 2),    # Pd^T.dO / dS^T.Q (TN)
    (256, 256, 192, False, True, 128, 1),
    (384, 128, 320, False, False, 128, 2),
    (256, 384, 256, True, False, 128, 1),
]
# x2-only tile codes (gemm_x2.hip X2Cfg): 257 = 256x128 BK 16, 130 = 128x128 BK 32 two stages; the
# fp32-operand reference runs the same block shape and K order (tile 256 / 128 resp. 129)
X2_CODES = [(512, 384, 512, False, True, 257, 256, 1), (512, 384, 512, False, False, 257, 256, 3),
            (512, 384, 512, True, False, 257, 256, 2), (256, 256, 256, False, True, 130, 128, 1),
            (384, 128, 320, False, False, 130, 128, 2), (256, 384, 256, True, False, 130, 128, 1),
            (512, 384, 512, False, True, 258, 256, 1), (512, 384, 512, False, False, 258, 256, 3),
            (512, 384, 512, True, False, 258, 256, 1), (512, 384, 512, False, True, 259, 256, 1),
            (512, 384, 512, False, False, 259, 256, 2), (512, 384, 512, True, False, 259, 256, 1),
            (512, 512, 256, False, True, 260, 256, 1), (512, 512, 512, False, False, 260, 256, 2),
            (512, 512, 256, True, False, 260, 256, 1),
            # ping-pong schedule (261 = 256x128 BK 32, 262 = 256x256 BK 16, 263 = 256x128 BK 16), incl.
            # K spans of 1 and 2 tiles (prologue / tail paths) and an empty split
            (512, 384, 512, False, True, 261, 256, 1), (512, 384, 512, False, False, 261, 256, 3),
            (512, 384, 512, True, False, 261, 256, 2), (512, 384, 64, False, True, 261, 256, 1),
            (512, 384, 32, False, False, 261, 256, 1), (512, 384, 96, True, False, 261, 256, 4),
            (512, 512, 256, False, True, 262, 256, 1), (512, 512, 512, False, False, 262, 256, 2),
            (512, 512, 256, True, False, 262, 256, 1), (512, 384, 512, False, True, 263, 256, 1),
            (512, 384, 512, False, False, 263, 256, 3), (512, 384, 48, True, False, 263, 256, 2)]


@pytest.mark.parametrize("M,N,Kd,ta,tb,tile,split", CASES)
def test_x2_gemm_bit_identical_to_bf16x3(M, N, Kd, ta, tb, tile, split):
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.randn(Kd, M, device="cuda", generator=g) if ta else torch.randn(M, Kd, device="cuda", generator=g)
    B = torch.randn(N, Kd, device="cuda", generator=g) if tb else torch.randn(Kd, N, device="cuda", generator=g)
    C_ref = torch.empty(split, M, N, device="cuda")
    K.gemm(A, B, C_ref, M, N, Kd, A.stride(0), B.stride(0), N, trans_a=ta, trans_b=tb, precision="bf16x3",
           tile=tile, split_k=split, slab_stride=M * N)
    A2, B2 = to_x2(A), to_x2(B)
    C = torch.full((split, M, N), float("nan"), device="cuda")
    K.gemm(A2, B2, C, M, N, Kd, A2.stride(0), B2.stride(0), N, trans_a=ta, trans_b=tb, precision="bf16x3",
           tile=tile, split_k=split, slab_stride=M * N)
    torch.cuda.synchronize()
    assert torch.equal(C, C_ref)
    ref = (A.double().T if ta else A.double()) @ (B.double().T if tb else B.double())
    err = (C.sum(0).double() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize("M,N,Kd,ta,tb,code,ref_tile,split", X2_CODES)
def test_x2_gemm_tile_codes(M, N, Kd, ta, tb, code, ref_tile, split):
    g = torch.Generator(device="cuda").manual_seed(7)
    A = torch.randn(Kd, M, device="cuda", generator=g) if ta else torch.randn(M, Kd, device="cuda", generator=g)
    B = torch.randn(N, Kd, device="cuda", generator=g) if tb else torch.randn(Kd, N, device="cuda", generator=g)
    A2, B2 = to_x2(A), to_x2(B)
    C = torch.full((split, M, N), float("nan"), device="cuda")
    K.gemm(A2, B2, C, M, N, Kd, A2.stride(0), B2.stride(0), N, trans_a=ta, trans_b=tb, precision="bf16x3",
           tile=code, split_k=split, slab_stride=M * N)
    torch.cuda.synchronize()
    ref = (A.double().T if ta else A.double()) @ (B.double().T if tb else B.double())
    err = (C.sum(0).double() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item()
    if split == 1:   # the same K order as the fp32-operand kernel with the same K step: bit-identical
        C_ref = torch.empty(M, N, device="cuda")
        K.gemm(A, B, C_ref, M, N, Kd, A.stride(0), B.stride(0), N, trans_a=ta, trans_b=tb, precision="bf16x3",
               tile=ref_tile)
        torch.cuda.synchronize()
        assert torch.equal(C[0], C_ref)


def test_x2_gemm_x2_output_and_views():
    """Strided views inside a wider x2 buffer (the QKV layout) and an x2 epilogue output."""
    g = torch.Generator(device="cuda").manual_seed(2)
    Np, dp = 512, 128
    QKV = torch.randn(Np, 3 * dp, device="cuda", generator=g)
    QKV2 = to_x2(QKV)
    Q2, K2 = QKV2[:, :2 * dp], QKV2[:, 2 * dp:4 * dp]
    S = torch.empty(Np, Np, device="cuda")
    S2 = torch.empty(Np, 2 * Np, device="cuda", dtype=torch.bfloat16)
    K.gemm(Q2, K2, S, Np, Np, dp, QKV2.stride(0), QKV2.stride(0), Np, trans_b=True, precision="bf16x3", tile=256,
           Cx2=S2, ldcx2=S2.stride(0))
    S_ref = torch.empty(Np, Np, device="cuda")
    K.gemm(QKV[:, :dp], QKV[:, dp:2 * dp], S_ref, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True,
           precision="bf16x3", tile=256)
    torch.cuda.synchronize()
    assert torch.equal(S, S_ref)
    assert torch.equal(S2, to_x2(S_ref))


def test_old_gemm_x2_output():
    """The fp32-operand kernels write x2 outputs too (QKV projection, dO)."""
    g = torch.Generator(device="cuda").manual_seed(3)
    M, N, Kd = 256, 192, 128
    A = torch.randn(M, Kd, device="cuda", generator=g)
    B = torch.randn(N, Kd, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    C2 = torch.empty(M, 2 * N, device="cuda", dtype=torch.bfloat16)
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=E.EPI_BIAS, bias=bias, alpha=0.5, scale_cols=64,
           precision="bf16x3", tile=64, Cx2=C2, ldcx2=2 * N)
    C2b = torch.empty(M, 2 * N, device="cuda", dtype=torch.bfloat16)
    K.gemm(A, B, None, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=E.EPI_BIAS, bias=bias, alpha=0.5, scale_cols=64,
           precision="bf16x3", tile=64, Cx2=C2b, ldcx2=2 * N)
    torch.cuda.synchronize()
    assert torch.equal(C2, to_x2(C))
    assert torch.equal(C2b, C2)


@pytest.mark.parametrize("N,p", [(1000, 0.5), (1000, 0.0), (300, 0.5)])
def test_softmax_x2_matches_signed_softmax(N, p):
    Np = 1024 if N > 512 else 384
    g = torch.Generator(device="cuda").manual_seed(4)
    S = torch.randn(Np, Np, device="cuda", generator=g) * 3
    seed = 12345
    Pd_signed = torch.empty(Np, Np, device="cuda")
    if p > 0:
        K.attn_softmax_fwd(S, Np, None, Pd_signed, Np, N, Np, N, Np, p, seed)
        Pd_ref = Pd_signed.clamp(min=0)
    else:
        K.attn_softmax_fwd(S, Np, Pd_signed, Pd_signed, Np, N, Np, N, Np, p, seed)
        Pd_ref = Pd_signed
    Pd2 = torch.empty(Np, 2 * Np, device="cuda", dtype=torch.bfloat16)
    rs = torch.empty(Np, 2, device="cuda")
    K.attn_softmax_x2_fwd(S, Np, Pd2, Pd2.stride(0), rs, N, Np, N, Np, p, seed)
    torch.cuda.synchronize()
    assert torch.equal(Pd2, to_x2(Pd_ref))
    m = S[:N, :N].max(1).values
    assert torch.equal(rs[:N, 0], m)
    ref_inv = 1.0 / torch.exp(S[:N, :N] - m[:, None]).sum(1)
    assert torch.allclose(rs[:N, 1], ref_inv, rtol=1e-5)
    assert (rs[N:] == 0).all()


@pytest.mark.parametrize("N,p", [(1000, 0.5), (1000, 0.0)])
def test_ds_recompute_epilogue_matches_signed(N, p):
    Np, dp = 1024, 128
    g = torch.Generator(device="cuda").manual_seed(5)
    S = torch.randn(Np, Np, device="cuda", generator=g) * 2
    S[N:] = 0
    seed = 777
    img = torch.empty(Np, Np, device="cuda")
    if p > 0:
        K.attn_softmax_fwd(S, Np, None, img, Np, N, Np, N, Np, p, seed)
    else:
        K.attn_softmax_fwd(S, Np, img, img, Np, N, Np, N, Np, p, seed)
    Pd2 = torch.empty(Np, 2 * Np, device="cuda", dtype=torch.bfloat16)
    rs = torch.empty(Np, 2, device="cuda")
    K.attn_softmax_x2_fwd(S, Np, Pd2, Pd2.stride(0), rs, N, Np, N, Np, p, seed)
    dO = torch.randn(Np, dp, device="cuda", generator=g)
    dO[N:] = 0
    V = torch.randn(Np, dp, device="cuda", generator=g)
    delta = torch.randn(Np, device="cuda", generator=g)
    delta[N:] = 0
    dS_ref = torch.empty(Np, Np, device="cuda")
    K.gemm(dO, V, dS_ref, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=E.EPI_ATTN_DS_SIGNED if p > 0 else E.EPI_ATTN_DS,
           aux0=img, aux1=img, rowvec=delta, ld_aux=Np, p_drop=p, precision="bf16x3", tile=128)
    dS2 = torch.empty(Np, 2 * Np, device="cuda", dtype=torch.bfloat16)
    dO2, V2 = to_x2(dO), to_x2(V)
    K.gemm(dO2, V2, None, Np, Np, dp, dO2.stride(0), V2.stride(0), Np, trans_b=True, epilogue=E.EPI_ATTN_DS_RECOMP,
           aux0=S, ld_aux=Np, rowvec=delta, rowstat=rs, m_valid=N, n_valid=N, p_drop=p, seed=seed,
           precision="bf16x3", tile=256, Cx2=dS2, ldcx2=dS2.stride(0))
    torch.cuda.synchronize()
    dS, _ = from_x2(dS2)
    scale = dS_ref.abs().max().item()
    assert (dS - dS_ref).abs().max().item() <= 1e-5 * scale
    assert (dS[N:] == 0).all() and (dS[:, N:] == 0).all()


@pytest.mark.parametrize("Np,Kd", [(512, 384), (1024, 64), (2304, 416)])
def test_x3_persistent_nt_kernel(Np, Kd):
    """gemm_x3.hip (tile code 301: persistent 256x128 blocks, 16x16x32 MFMAs, ping-pong waves) on
    x2 operands: S = Q.K^T and the signed-image dS epilogue against float64 (bf16x3 accuracy)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(Np, Kd, device="cuda", generator=g)
    B = torch.randn(Np, Kd, device="cuda", generator=g)
    A2, B2 = to_x2(A), to_x2(B)
    C = torch.full((Np, Np), float("nan"), device="cuda")
    K.gemm(A2, B2, C, Np, Np, Kd, A2.stride(0), B2.stride(0), Np, trans_b=True, precision="bf16x3", tile=301)
    ref = A.double() @ B.double().t()
    assert ((C.double() - ref).abs().max() / ref.abs().max()).item() < 3e-5
    img = torch.rand(Np, Np, device="cuda", generator=g) * 1e-3
    img = torch.where(torch.rand(Np, Np, device="cuda", generator=g) < 0.5, -img, img)
    delta = torch.randn(Np, device="cuda", generator=g)
    C.fill_(float("nan"))
    K.gemm(A2, B2, C, Np, Np, Kd, A2.stride(0), B2.stride(0), Np, trans_b=True, epilogue=E.EPI_ATTN_DS_SIGNED,
           aux0=img, rowvec=delta, ld_aux=Np, p_drop=0.5, precision="bf16x3", tile=301)
    x = img.double()
    dl = delta.double()[:, None]
    refd = torch.where(x < 0, x * dl, x * (ref - 0.5 * dl))
    assert ((C.double() - refd).abs().max() / refd.abs().max()).item() < 3e-5
