"""U2GNN_PREC_BF16X6 (ABI v17): the three-plane split-bf16 GEMM of the "fwd6" policy's forward products.

x = hi + mid + lo with every plane a bf16 and both residuals exact in fp32, so the planes hold every bit of an
fp32 operand; the kernel forms hh + hm + mh + hl + lh + mm (dropping terms below 2^-27 of the product) on the bf16
matrix cores with fp32 accumulation.  Its error must therefore be at the fp32 MFMA kernel's level (the k-ordered
fp32 fma chain of the reference's arithmetic), an order of magnitude below bf16x3's -- checked against float64 on
every tile and forward layout, the fused epilogues, ragged split-K, and operands exactly representable in bf16
(where the product is exact)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import _lib  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402
from u2gnn_hip._lib import U2GNNNativeError  # noqa: E402

DEV = "cuda"


def _mk(*s, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*s, generator=g).to(DEV)


def _err(C, ref):
    """max |C - ref| / max |ref| (float64)"""
    return ((C.double() - ref).abs().max() / ref.abs().max()).item()


def _run(prec, A, B, M, N, Kd, ta, tb, tile, **kw):
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, A.shape[1], B.shape[1], N, trans_a=ta, trans_b=tb, tile=tile, precision=prec, **kw)
    return C


@pytest.mark.parametrize("tile", [64, 128, 256, 129, 0])
@pytest.mark.parametrize("layout", ["NT", "NN"])
def test_x6_matches_fp32_accuracy(tile, layout):
    M, N, Kd = 512, 384, 368        # K a multiple of the 16-deep step, not of 32
    tb = layout[1] == "T"
    A = _mk(M, Kd, seed=21)
    B = _mk(N, Kd, seed=22) if tb else _mk(Kd, N, seed=22)
    ref = A.double() @ (B.t() if tb else B).double()
    e6 = _err(_run("bf16x6", A, B, M, N, Kd, False, tb, tile), ref)
    e32 = _err(_run("fp32", A, B, M, N, Kd, False, tb, 64 if tile in (0, 64) else 128), ref)
    assert e6 < 1e-6, e6
    assert e6 <= 2.0 * e32 + 1e-7, (e6, e32)
    if Kd % 32 == 0 or tile == 129:
        e3 = _err(_run("bf16x3", A, B, M, N, Kd, False, tb, tile), ref)
        assert e6 * 5 < e3, (e6, e3)


def test_x6_exact_on_bf16_representable_operands():
    """operands with 8 significant bits: every product is exact and the sums are the fp32 sums of exact terms"""
    M, N, Kd = 128, 128, 64
    A = (torch.randint(-64, 64, (M, Kd), device=DEV).float() / 8)
    B = (torch.randint(-64, 64, (N, Kd), device=DEV).float() / 16)
    C = _run("bf16x6", A, B, M, N, Kd, False, True, 64)
    assert torch.equal(C, A @ B.t())   # integer-valued partial sums: exact in fp32


def test_x6_fp32_operand_planes_are_exact():
    """an operand of full fp32 precision against the identity: hi + mid + lo reproduces it bit for bit"""
    M = N = Kd = 128
    A = torch.eye(M, device=DEV)
    B = _mk(Kd, N, seed=5) * 1e3
    C = _run("bf16x6", A, B, M, N, Kd, False, False, 64)
    assert torch.equal(C, B)


@pytest.mark.parametrize("tile", [64, 128])
def test_x6_epilogues(tile):
    M, N, Kd = 256, 256, 192
    A, B = _mk(M, Kd, seed=5), _mk(N, Kd, seed=6)
    bias, R = _mk(N, seed=7), _mk(M, N, seed=8)
    acc = A.double() @ B.t().double()
    C = _run("bf16x6", A, B, M, N, Kd, False, True, tile, epilogue=_lib.EPI_BIAS, bias=bias, alpha=0.5, scale_cols=64)
    ref = acc + bias.double()
    ref[:, :64] *= 0.5
    assert _err(C, ref) < 1e-6
    p, seed = 0.5, 4321
    mask = K.dropout_mask(seed, M, N, p).double()
    C = _run("bf16x6", A, B, M, N, Kd, False, True, tile, epilogue=_lib.EPI_BIAS_DROP_RESID, bias=bias, aux0=R,
             ld_aux=N, p_drop=p, seed=seed)
    assert _err(C, R.double() + (acc + bias.double()) * mask * 2) < 1e-6
    C = _run("bf16x6", A, B, M, N, Kd, False, True, tile, epilogue=_lib.EPI_BIAS_RELU_DROP, bias=bias, p_drop=p,
             seed=seed)
    assert _err(C, torch.relu(acc + bias.double()) * mask * 2) < 1e-6
    C2 = R.clone()
    K.gemm(A, B, C2, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ACCUM, precision="bf16x6", tile=tile)
    assert _err(C2, R.double() + acc) < 1e-6


def test_x6_rowstat_epilogue_equals_store():
    """S = Q K^T with the softmax row partials (the fused attention's QK^T): the stored scores are the STORE
    epilogue's bits, masked keys -inf"""
    Np, dp, n_valid = 512, 128, 500
    Q, Kt = _mk(Np, dp, seed=41), _mk(Np, dp, seed=42)
    S = torch.empty(Np, Np, device=DEV)
    rp = torch.empty(Np, 2 * (Np // 32), device=DEV)
    K.gemm(Q, Kt, S, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_STORE_ROWSTAT, rowpart=rp,
           n_valid=n_valid, precision="bf16x6", tile=128)
    S0 = _run("bf16x6", Q, Kt, Np, Np, dp, False, True, 128)
    assert torch.equal(S[:, :n_valid], S0[:, :n_valid])
    assert torch.isinf(S[:, n_valid:]).all() and (S[:, n_valid:] < 0).all()


@pytest.mark.parametrize("Kd,split,tile", [(368, 4, 128), (96, 8, 64), (336, 5, 256)])
def test_x6_ragged_split_k(Kd, split, tile):
    M, N = 256, 128
    A, B = _mk(M, Kd, seed=31), _mk(Kd, N, seed=32)
    slabs = torch.full((split, M, N), float("nan"), device=DEV)
    K.gemm(A, B, slabs, M, N, Kd, Kd, N, N, split_k=split, slab_stride=M * N, tile=tile, precision="bf16x6")
    assert torch.isfinite(slabs).all()
    assert _err(slabs.sum(0), A.double() @ B.double()) < 1e-6


def test_x6_clamped_signed_image_operand():
    """P.V over the signed probability image (negatives staged as 0), the unfused forward's P.V product"""
    M, N, Kd = 256, 128, 256
    X = _mk(M, Kd, seed=51)
    V = _mk(Kd, N, seed=52)
    C = _run("bf16x6", X, V, M, N, Kd, False, False, 128, clamp_a=True)
    assert _err(C, X.clamp_min(0).double() @ V.double()) < 1e-6


def test_x6_refuses_the_backward_layouts_and_epilogues():
    M = N = Kd = 128
    A, B = _mk(Kd, M, seed=1), _mk(Kd, N, seed=2)
    C = torch.empty(M, N, device=DEV)
    with pytest.raises(U2GNNNativeError):   # A transposed: the weight-gradient layout
        K.gemm(A, B, C, M, N, Kd, M, N, N, trans_a=True, precision="bf16x6")
    with pytest.raises(U2GNNNativeError):   # a backward epilogue
        K.gemm(A, B, C, M, N, Kd, Kd, N, N, epilogue=_lib.EPI_RELU_DROP_BWD, aux0=C, ld_aux=N, precision="bf16x6")
    with pytest.raises(U2GNNNativeError):   # not a multiple of the 16-deep K step
        K.gemm(A, B, C, M, N, 120, Kd, N, N, precision="bf16x6")
