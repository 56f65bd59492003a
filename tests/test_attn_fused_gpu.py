"""The fused node-axis attention forward (ABI v10, attn_fused.hip): the QK^T GEMM's EPI_STORE_ROWSTAT
row partials and u2gnn_attn_softmax_pv, each against a plain torch
reference (fp32 / fp64) of softmax(S) -> dropout -> P.V as torch's MultiheadAttention forms it
(pytorch_U2GNN_Sup.py:19-21,35)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import _lib  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402

DEV = "cuda"


def _mk(*s, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*s, generator=g) * scale).to(DEV)


def _ref_rowstat(S, N, Np):
    """(max, 1/sum exp(S - max)) over the first N columns of rows < N; (0, 0) below."""
    s = S[:N, :N].double()
    m = s.max(dim=1).values
    l = torch.exp(s - m[:, None]).sum(dim=1)
    out = torch.zeros(Np, 2, dtype=torch.float64, device=DEV)
    out[:N, 0], out[:N, 1] = m, 1.0 / l
    return out


@pytest.mark.parametrize("Np,N,dp,tile", [(256, 230, 64, 256), (1280, 1100, 384, 128), (512, 512, 128, 256),
                                          (4864, 4776, 384, 256), (384, 70, 64, 128)])
@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
def test_store_rowstat_epilogue(Np, N, dp, tile, prec):
    """S is bitwise the plain STORE result over the N real keys (-inf beyond); each 64-column group carries (max, sum exp(S - max)) of its
    columns < N, (-inf, 0) when it has none."""
    QKV = _mk(Np, 3 * dp, seed=3, scale=0.3)
    Q, Kt = QKV[:, :dp], QKV[:, dp:2 * dp]
    S0 = torch.empty(Np, Np, device=DEV)
    K.gemm(Q, Kt, S0, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True, precision=prec, tile=tile, alpha=0.7)
    S = torch.full((Np, Np), float("nan"), device=DEV)
    rp = torch.full((Np, 2 * (Np // 32)), float("nan"), device=DEV)
    K.gemm(Q, Kt, S, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True, precision=prec, tile=tile, alpha=0.7,
           epilogue=_lib.EPI_STORE_ROWSTAT, rowpart=rp, n_valid=N)
    torch.cuda.synchronize()
    assert torch.equal(S[:, :N], S0[:, :N])
    assert torch.isneginf(S[:, N:]).all()   # masked keys: exp(-inf) = 0 downstream
    G = Np // 64
    pairs = rp[:, :2 * G].view(Np, G, 2)[:N].double()
    s = S0[:N].double().view(N, G, 64)
    col = torch.arange(Np, device=DEV).view(G, 64)
    valid = (col < N)[None].expand(N, G, 64)
    sm = torch.where(valid, s, torch.full_like(s, float("-inf")))
    m = sm.max(dim=2).values
    l = torch.where(valid, torch.exp(sm - m[..., None].clamp_min(-1e30)), torch.zeros_like(s)).sum(dim=2)
    live = valid.any(dim=2)
    assert torch.equal(pairs[..., 0][live], m[live])
    assert ((pairs[..., 1][live] - l[live]).abs() / l[live]).max().item() < 2e-6
    if (~live).any():
        assert torch.isneginf(pairs[..., 0][~live]).all() and (pairs[..., 1][~live] == 0).all()


def _partials(S, N, Np):
    """EPI_STORE_ROWSTAT-shaped partials of S (float32 [Np, 2 * Np/32]: (max, sum exp) per 64-column group
    over the columns < N, (-inf, 0) for a group without any), computed in fp64."""
    G = Np // 64
    rp = torch.zeros(Np, 2 * (Np // 32), device=DEV)
    s = S.double().view(Np, G, 64)
    col = torch.arange(Np, device=DEV).view(G, 64)
    valid = (col < N)[None].expand(Np, G, 64)
    sm = torch.where(valid, s, torch.full_like(s, float("-inf")))
    m = sm.max(dim=2).values
    l = torch.where(valid, torch.exp(sm - m[..., None].clamp_min(-1e30)), torch.zeros_like(s)).sum(dim=2)
    rp[:, :2 * G].view(Np, G, 2)[..., 0] = m.float()
    rp[:, :2 * G].view(Np, G, 2)[..., 1] = l.float()
    return rp


def _qkv2(V, Np, dp):
    """x2 image of an in-projection output whose V block is V (Q, K blocks arbitrary)."""
    QKV = _mk(Np, 3 * dp, seed=11)
    QKV[:, 2 * dp:] = V
    Q2 = torch.empty(Np, 6 * dp, device=DEV, dtype=torch.bfloat16)
    K.split_x2(QKV, 3 * dp, Q2, 6 * dp, Np, 3 * dp)
    return Q2


@pytest.mark.parametrize("Np,N,dp", [(256, 230, 64), (128, 100, 384), (1280, 1100, 128), (512, 500, 384),
                                     (2048, 1999, 192), (4864, 4776, 384), (384, 257, 256), (640, 640, 320)])
@pytest.mark.parametrize("p", [0.5, 0.0])
@pytest.mark.parametrize("prec,tol", [("bf16x3", 2e-5), ("bf16", 2e-2)])
def test_softmax_pv(Np, N, dp, p, prec, tol):
    """O = dropout(softmax(S)) V over the N real rows / keys (fp64 reference), the signed image
    (sign bit = keep bit of the dropout hash, magnitude P/(1-p) kept, P dropped, zeros in the padding),
    and S / Pd aliasing gives the same bits."""
    seed = 4242
    S = _mk(Np, Np, seed=7, scale=2.0)
    S[:, N:] = float("-inf")   # as EPI_STORE_ROWSTAT leaves the masked keys
    V = _mk(Np, dp, seed=9)
    rp = _partials(S, N, Np)
    rs = _ref_rowstat(S, N, Np)
    Q2 = _qkv2(V, Np, dp)
    ws = torch.empty(K.attn_softmax_pv_ws_floats(N, Np, dp), device=DEV)
    Pd = torch.full((Np, Np), float("nan"), device=DEV)
    O = torch.full((Np, dp), float("nan"), device=DEV)
    K.attn_softmax_pv(S, Np, rp, Np // 64, Q2, 6 * dp, dp, Pd, Np, O, dp, ws, N, Np, p, seed, precision=prec)
    # in place over the scores (how the encoder layer runs it)
    X = S.clone()
    O2 = torch.full((Np, dp), float("nan"), device=DEV)
    K.attn_softmax_pv(X, Np, rp, Np // 64, Q2, 6 * dp, dp, X, Np, O2, dp, ws, N, Np, p, seed, precision=prec)
    torch.cuda.synchronize()
    assert torch.equal(X, Pd) and torch.equal(O2, O)

    s = S[:N, :N].double()
    P = torch.exp(s - rs[:N, 0:1]) * rs[:N, 1:2]
    keep = K.dropout_mask(seed, Np, Np, p).bool()[:N, :N] if p > 0 else torch.ones_like(P, dtype=torch.bool)
    img = torch.where(keep, P / (1.0 - p), -P)
    O_ref = img.clamp_min(0) @ V[:N].double()
    assert torch.equal(torch.signbit(Pd[:N, :N]), ~keep)
    assert ((Pd[:N, :N].double() - img).abs().max() / img.abs().max()).item() < 2e-6
    assert (Pd[N:] == 0).all() and (Pd[:, N:] == 0).all()
    err = ((O[:N].double() - O_ref).abs().max() / O_ref.abs().max()).item()
    assert err < tol, err
    assert (O[N:] == 0).all()


def test_softmax_pv_rejects_bad_shapes():
    Np, N, dp = 256, 200, 64
    S = torch.zeros(Np, Np, device=DEV)
    rp = torch.zeros(Np, 2 * (Np // 32), device=DEV)
    Q2 = torch.zeros(Np, 6 * dp, device=DEV, dtype=torch.bfloat16)
    O = torch.zeros(Np, dp, device=DEV)
    ws = torch.zeros(K.attn_softmax_pv_ws_floats(N, Np, dp), device=DEV)
    G = Np // 64
    with pytest.raises(_lib.U2GNNNativeError):   # dp not a multiple of 64
        K.attn_softmax_pv(S, Np, rp, G, Q2, 6 * dp, 96, S, Np, O, dp, ws, N, Np, 0.5, 1)
    with pytest.raises(_lib.U2GNNNativeError):   # workspace too small
        K.attn_softmax_pv(S, Np, rp, G, Q2, 6 * dp, dp, S, Np, O, dp, ws[:16], N, Np, 0.5, 1)
    with pytest.raises(_lib.U2GNNNativeError):   # rows_pad not a multiple of 128
        K.attn_softmax_pv(S, Np, rp, G, Q2, 6 * dp, dp, S, Np, O, dp, ws, N, 200, 0.5, 1)
    with pytest.raises(_lib.U2GNNNativeError):   # odd group count
        K.attn_softmax_pv(S, Np, rp, 3, Q2, 6 * dp, dp, S, Np, O, dp, ws, N, Np, 0.5, 1)
    with pytest.raises(_lib.U2GNNNativeError):   # fp32 is the split path's precision
        K.attn_softmax_pv(S, Np, rp, G, Q2, 6 * dp, dp, S, Np, O, dp, ws, N, Np, 0.5, 1, precision="fp32")


@pytest.mark.parametrize("Np,N,dp", [(256, 230, 64), (128, 100, 384), (1280, 1100, 128), (512, 500, 384),
                                     (2048, 1999, 192), (4864, 4776, 384), (384, 257, 256), (640, 640, 320)])
@pytest.mark.parametrize("p", [0.5, 0.0])
def test_softmax_pv_bf16x6(Np, N, dp, p):
    """ABI v17 BF16X6: V straight from the fp32 in-projection output (ldq2 = 3 dp floats), P and V split three
    ways in registers: O within fp32 rounding of the fp64 reference (an order below bf16x3's), and the signed
    image bit for bit the bf16x3 kernel's (the same P and keep decisions)."""
    seed = 4242
    S = _mk(Np, Np, seed=7, scale=2.0)
    S[:, N:] = float("-inf")
    V = _mk(Np, dp, seed=9)
    rp = _partials(S, N, Np)
    rs = _ref_rowstat(S, N, Np)
    QKV = _mk(Np, 3 * dp, seed=11)
    QKV[:, 2 * dp:] = V
    ws = torch.empty(K.attn_softmax_pv_ws_floats(N, Np, dp), device=DEV)
    X6, O6 = S.clone(), torch.full((Np, dp), float("nan"), device=DEV)
    K.attn_softmax_pv(X6, Np, rp, Np // 64, QKV, 3 * dp, dp, X6, Np, O6, dp, ws, N, Np, p, seed, precision="bf16x6")
    X3, O3 = S.clone(), torch.full((Np, dp), float("nan"), device=DEV)
    K.attn_softmax_pv(X3, Np, rp, Np // 64, _qkv2(V, Np, dp), 6 * dp, dp, X3, Np, O3, dp, ws, N, Np, p, seed,
                      precision="bf16x3")
    torch.cuda.synchronize()
    assert torch.equal(X6, X3)
    s = S[:N, :N].double()
    P = torch.exp(s - rs[:N, 0:1]) * rs[:N, 1:2]
    keep = K.dropout_mask(seed, Np, Np, p).bool()[:N, :N] if p > 0 else torch.ones_like(P, dtype=torch.bool)
    img = torch.where(keep, P / (1.0 - p), -P)
    # the reference from the kernel's own fp32 image (P carries exp2 / rounding of its own): the products' error only
    O_ref = X6[:N, :N].double().clamp_min(0) @ V[:N].double()
    O_ref_p = img.clamp_min(0) @ V[:N].double()
    e6 = ((O6[:N].double() - O_ref).abs().max() / O_ref.abs().max()).item()
    e3 = ((O3[:N].double() - O_ref).abs().max() / O_ref.abs().max()).item()
    assert e6 < 1e-6, e6
    assert e6 * 4 < e3, (e6, e3)
    assert ((O6[:N].double() - O_ref_p).abs().max() / O_ref_p.abs().max()).item() < 2e-6
    assert (O6[N:] == 0).all()


def x2h(X, scale_exp=6):
    """The f16x3 x2 image of fp32 X (u2gnn_hip.h U2GNN_H3_X2_EXP): per 8 columns fp16 hi then lo of 2^6 X."""
    x = X.float() * 2.0 ** scale_exp
    hi = x.half()
    lo = (x - hi.float()).half()
    R, C = X.shape
    img = torch.stack([hi.view(R, C // 8, 8), lo.view(R, C // 8, 8)], dim=2).reshape(R, 2 * C)
    return img.view(torch.int16).view(torch.bfloat16)


@pytest.mark.parametrize("Np,N,dp", [(256, 230, 64), (128, 100, 384), (1280, 1100, 128), (512, 500, 384),
                                     (2048, 1999, 192), (4864, 4776, 384), (384, 257, 256), (640, 640, 320)])
@pytest.mark.parametrize("p", [0.5, 0.0])
def test_softmax_pv_f16x3(Np, N, dp, p):
    """ABI v18 F16X3: V as x2 rows of fp16 planes of 2^6 V (the in-projection's f16x3 x2 output), P pre-scaled by
    2^h3_prob_exp(p) and split in registers: O well below bf16x3's error against the fp64 product of the kernel's
    own image, and the signed image bit for bit the bf16x3 kernel's (the same P and keep decisions)."""
    seed = 4243
    S = _mk(Np, Np, seed=17, scale=2.0)
    S[:, N:] = float("-inf")
    V = _mk(Np, dp, seed=19)
    rp = _partials(S, N, Np)
    QKV = _mk(Np, 3 * dp, seed=21)
    QKV[:, 2 * dp:] = V
    ws = torch.empty(K.attn_softmax_pv_ws_floats(N, Np, dp), device=DEV)
    Xh, Oh = S.clone(), torch.full((Np, dp), float("nan"), device=DEV)
    K.attn_softmax_pv(Xh, Np, rp, Np // 64, x2h(QKV), 6 * dp, dp, Xh, Np, Oh, dp, ws, N, Np, p, seed, precision="f16x3")
    X3, O3 = S.clone(), torch.full((Np, dp), float("nan"), device=DEV)
    K.attn_softmax_pv(X3, Np, rp, Np // 64, _qkv2(V, Np, dp), 6 * dp, dp, X3, Np, O3, dp, ws, N, Np, p, seed,
                      precision="bf16x3")
    torch.cuda.synchronize()
    assert torch.equal(Xh, X3)
    O_ref = Xh[:N, :N].double().clamp_min(0) @ V[:N].double()
    eh = ((Oh[:N].double() - O_ref).abs().max() / O_ref.abs().max()).item()
    e3 = ((O3[:N].double() - O_ref).abs().max() / O_ref.abs().max()).item()
    assert eh < 4e-6, eh
    assert eh * 4 < e3, (eh, e3)
    assert (Oh[N:] == 0).all()
