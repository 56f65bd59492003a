"""U2GNN_PREC_F16X3 (ABI v18): the two-plane fp16 split GEMM of the "fwdh" policy's forward products.

x = hi + lo with hi = fp16(x), lo = fp16(x - hi) (the residual exact in fp32): 22 significant bits per operand;
the kernel forms hh + hl + lh on the fp16 matrix cores with fp32 accumulation (the dropped lo.lo term is below
2^-22 of the product).  Its error must sit between bf16x6's (fp32-class) and bf16x3's (2^-16 planes): checked
against float64 on every tile and forward layout, the fused epilogues, ragged split-K, the clamped signed image,
operands exactly representable in fp16 (exact products), small-magnitude operands and the documented range limit
(|x| * 2^h3_exp >= 65520 overflows hi to inf: a loud failure, never a silently wrong number).  The operand
pre-scales (h3_exp, ABI v18; default 2^6 each, the layer executor's) keep lo out of fp16's subnormals: checked
on the probability image, whose entries are ~1/N."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import _lib  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402
from u2gnn_hip._lib import U2GNNNativeError  # noqa: E402

DEV = "cuda"
TOL = 4e-6   # max|C - ref| / max|ref| against float64 (bf16x3 on the same operands: ~1e-5 .. 4e-5)


def _mk(*s, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*s, generator=g).to(DEV)


def _err(C, ref):
    return ((C.double() - ref).abs().max() / ref.abs().max()).item()


def _run(prec, A, B, M, N, Kd, ta, tb, tile, **kw):
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, M, N, Kd, A.shape[1], B.shape[1], N, trans_a=ta, trans_b=tb, tile=tile, precision=prec, **kw)
    return C


@pytest.mark.parametrize("tile", [64, 128, 256, 129, 0])
@pytest.mark.parametrize("layout", ["NT", "NN"])
def test_h3_between_x6_and_x3(tile, layout):
    M, N, Kd = 512, 384, 384
    tb = layout[1] == "T"
    A = _mk(M, Kd, seed=21)
    B = _mk(N, Kd, seed=22) if tb else _mk(Kd, N, seed=22)
    ref = A.double() @ (B.t() if tb else B).double()
    eh = _err(_run("f16x3", A, B, M, N, Kd, False, tb, tile), ref)
    e3 = _err(_run("bf16x3", A, B, M, N, Kd, False, tb, tile), ref)
    assert eh < TOL, eh
    assert eh * 8 < e3, (eh, e3)


def test_h3_exact_on_fp16_representable_operands():
    """operands with 11 significant bits: lo = 0, every product exact, integer-valued sums exact in fp32"""
    M, N, Kd = 128, 128, 64
    A = (torch.randint(-1024, 1024, (M, Kd), device=DEV).float() / 64)
    B = (torch.randint(-1024, 1024, (N, Kd), device=DEV).float() / 128)
    C = _run("f16x3", A, B, M, N, Kd, False, True, 64)
    assert torch.equal(C, A @ B.t())


def test_h3_identity_keeps_22_bits():
    """an fp32 operand against the identity comes back as hi + lo: within 2^-22 of every element"""
    M = N = Kd = 128
    A = torch.eye(M, device=DEV)
    B = _mk(Kd, N, seed=5) * 1e3
    C = _run("f16x3", A, B, M, N, Kd, False, False, 64, h3_exp=(0, 0))
    assert ((C - B).abs() <= B.abs() * 2.0 ** -21).all()


def test_h3_small_magnitude_operands():
    """xavier-scale weights"""
    M, N, Kd = 256, 256, 384
    A = _mk(M, Kd, seed=61)
    W = _mk(N, Kd, seed=62) * 0.05
    ref = A.double() @ W.t().double()
    assert _err(_run("f16x3", A, W, M, N, Kd, False, True, 64), ref) < TOL


def test_h3_overflow_is_loud():
    M = N = Kd = 64
    A = _mk(M, Kd, seed=7)
    A[3, 5] = 1e5
    B = _mk(N, Kd, seed=8)
    C = _run("f16x3", A, B, M, N, Kd, False, True, 64)
    assert not torch.isfinite(C[3]).any() and torch.isfinite(C[:3]).all()


@pytest.mark.parametrize("tile", [64, 128])
def test_h3_epilogues(tile):
    M, N, Kd = 256, 256, 192
    A, B = _mk(M, Kd, seed=5), _mk(N, Kd, seed=6)
    bias, R = _mk(N, seed=7), _mk(M, N, seed=8)
    acc = A.double() @ B.t().double()
    C = _run("f16x3", A, B, M, N, Kd, False, True, tile, epilogue=_lib.EPI_BIAS, bias=bias, alpha=0.5, scale_cols=64)
    ref = acc + bias.double()
    ref[:, :64] *= 0.5
    assert _err(C, ref) < TOL
    p, seed = 0.5, 4321
    mask = K.dropout_mask(seed, M, N, p).double()
    C = _run("f16x3", A, B, M, N, Kd, False, True, tile, epilogue=_lib.EPI_BIAS_DROP_RESID, bias=bias, aux0=R,
             ld_aux=N, p_drop=p, seed=seed)
    assert _err(C, R.double() + (acc + bias.double()) * mask * 2) < TOL
    C = _run("f16x3", A, B, M, N, Kd, False, True, tile, epilogue=_lib.EPI_BIAS_RELU_DROP, bias=bias, p_drop=p,
             seed=seed)
    assert _err(C, torch.relu(acc + bias.double()) * mask * 2) < TOL
    C2 = R.clone()
    K.gemm(A, B, C2, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_ACCUM, precision="f16x3", tile=tile)
    assert _err(C2, R.double() + acc) < TOL


def test_h3_rowstat_epilogue_equals_store():
    Np, dp, n_valid = 512, 128, 500
    Q, Kt = _mk(Np, dp, seed=41), _mk(Np, dp, seed=42)
    S = torch.empty(Np, Np, device=DEV)
    rp = torch.empty(Np, 2 * (Np // 32), device=DEV)
    K.gemm(Q, Kt, S, Np, Np, dp, dp, dp, Np, trans_b=True, epilogue=_lib.EPI_STORE_ROWSTAT, rowpart=rp,
           n_valid=n_valid, precision="f16x3", tile=128)
    S0 = _run("f16x3", Q, Kt, Np, Np, dp, False, True, 128)
    assert torch.equal(S[:, :n_valid], S0[:, :n_valid])
    assert torch.isinf(S[:, n_valid:]).all() and (S[:, n_valid:] < 0).all()


@pytest.mark.parametrize("Kd,split,tile", [(384, 4, 128), (96, 8, 64), (352, 5, 256)])
def test_h3_ragged_split_k(Kd, split, tile):
    M, N = 256, 128
    A, B = _mk(M, Kd, seed=31), _mk(Kd, N, seed=32)
    slabs = torch.full((split, M, N), float("nan"), device=DEV)
    K.gemm(A, B, slabs, M, N, Kd, Kd, N, N, split_k=split, slab_stride=M * N, tile=tile, precision="f16x3")
    assert torch.isfinite(slabs).all()
    assert _err(slabs.sum(0), A.double() @ B.double()) < TOL


def test_h3_clamped_signed_image_operand():
    """P.V over the signed probability image (negatives staged as 0), probabilities down to ~1e-9"""
    M, N, Kd = 256, 128, 256
    X = torch.softmax(_mk(M, Kd, seed=51) * 4, dim=1) * torch.where(_mk(M, Kd, seed=53) > 0, 2.0, -1.0)
    V = _mk(Kd, N, seed=52)
    C = _run("f16x3", X, V, M, N, Kd, False, False, 128, clamp_a=True)
    assert _err(C, X.clamp_min(0).double() @ V.double()) < TOL


@pytest.mark.parametrize("N_keys", [1024, 4096])
def test_h3_probability_image_needs_its_prescale(N_keys):
    """P.V with softmax rows of ~N_keys entries ~1/N_keys: unscaled, lo is subnormal and the product loses bits
    (~2^-12 per entry); with the executor's pre-scale 2^h3_prob_exp(p) it is at the f16x3 level"""
    M, N = 256, 128
    P = torch.softmax(_mk(M, N_keys, seed=71), dim=1) * 2.0   # kept entries / (1 - p), p = 0.5
    V = _mk(N_keys, N, seed=72)
    ref = P.double() @ V.double()
    e_scaled = _err(_run("f16x3", P, V, M, N, N_keys, False, False, 128, h3_exp=(K.h3_prob_exp(0.5), K.H3_EXP)), ref)
    e_plain = _err(_run("f16x3", P, V, M, N, N_keys, False, False, 128, h3_exp=(0, 0)), ref)
    assert e_scaled < TOL, e_scaled
    assert e_scaled * 4 < e_plain, (e_scaled, e_plain)
    assert K.h3_prob_exp(0.0) == 15 and K.h3_prob_exp(0.5) == 14 and K.h3_prob_exp(0.9) == 11


def test_h3_prescale_arguments_checked():
    M = N = Kd = 64
    A, B = _mk(M, Kd, seed=1), _mk(N, Kd, seed=2)
    C = torch.empty(M, N, device=DEV)
    with pytest.raises(U2GNNNativeError):   # outside [-24, 24]
        K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, precision="f16x3", h3_exp=(25, 0))
    with pytest.raises(U2GNNNativeError):   # pre-scales belong to f16x3 only
        K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, precision="bf16x3", h3_exp=(6, 6))


def test_h3_refuses_the_backward_layouts_and_epilogues():
    M = N = Kd = 128
    A, B = _mk(Kd, M, seed=1), _mk(Kd, N, seed=2)
    C = torch.empty(M, N, device=DEV)
    with pytest.raises(U2GNNNativeError):   # A transposed: the weight-gradient layout
        K.gemm(A, B, C, M, N, Kd, M, N, N, trans_a=True, precision="f16x3")
    with pytest.raises(U2GNNNativeError):   # a backward epilogue
        K.gemm(A, B, C, M, N, Kd, Kd, N, N, epilogue=_lib.EPI_RELU_DROP_BWD, aux0=C, ld_aux=N, precision="f16x3")
    with pytest.raises(U2GNNNativeError):   # not a multiple of the 32-deep K step
        K.gemm(A, B, C, M, N, 112, Kd, N, N, precision="f16x3")


def test_h3_x2_output_is_fp16_planes_of_scaled_result():
    """with precision f16x3 the x2 output (Cx2) holds fp16 hi / lo of 2^U2GNN_H3_X2_EXP * C (the f16x3 fused
    softmax.P.V's V operand), bit for bit the planes of the stored C; columns below cx2_col0 untouched"""
    from test_attn_fused_gpu import x2h
    M, N, Kd = 256, 192, 128
    A, B = _mk(M, Kd, seed=81), _mk(N, Kd, seed=82)
    bias = _mk(N, seed=83)
    C = torch.empty(M, N, device=DEV)
    Cx2 = torch.zeros(M, 2 * N, device=DEV, dtype=torch.bfloat16)
    K.gemm(A, B, C, M, N, Kd, Kd, Kd, N, trans_b=True, epilogue=_lib.EPI_BIAS, bias=bias, precision="f16x3", tile=64,
           Cx2=Cx2, ldcx2=2 * N, cx2_col0=64)
    ref = x2h(C)
    assert torch.equal(Cx2[:, 128:].view(torch.int16), ref[:, 128:].view(torch.int16))
    assert (Cx2[:, :128].view(torch.int16) == 0).all()
