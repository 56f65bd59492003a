"""Small-width in-projection + node attention (u2gnn_attn_small_fwd / _bwd, csrc/small_layer.hip; d <= 32: the UnSup
encoders C3 / C5 and MUTAG) against a float64 torch restatement of the reference's MHA core on the same dropout
masks (pytorch_U2GNN_UnSup.py:37-40,57: q, k, v = x W_in^T + b_in with q scaled by 1/sqrt(d), softmax over the N
keys, dropout(0.5) on the probabilities with 1/(1-p) scaling, times V; the backward through torch autograd, down
to the in-projection's outputs and the layer input).  Tolerance 2e-5 of each tensor's scale (the kernels run
exact fp32); padding rows / columns must come out as exact zeros."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(N, d, seed):
    """-> Np, dp, X [Np, dp], W_in [3 dp, dp], b_in [3 dp] (padded, real blocks random), dO [Np, dp]."""
    from u2gnn_hip.engine import row_pad
    Np, dp = row_pad(N), 64
    g = torch.Generator(device=DEV).manual_seed(seed)
    X = torch.zeros(Np, dp, device=DEV)
    X[:N, :d] = torch.randn(N, d, device=DEV, generator=g)
    W = torch.zeros(3 * dp, dp, device=DEV)
    b = torch.zeros(3 * dp, device=DEV)
    for blk in range(3):
        W[blk * dp:blk * dp + d, :d] = torch.randn(d, d, device=DEV, generator=g) / math.sqrt(d)
        b[blk * dp:blk * dp + d] = 0.1 * torch.randn(d, device=DEV, generator=g)
    dO = torch.zeros(Np, dp, device=DEV)
    dO[:N, :d] = torch.randn(N, d, device=DEV, generator=g)
    return Np, dp, X, W, b, dO


def _ref(X, W, b, dO, N, d, dp, keep, p):
    x = X[:N, :d].double().cpu().requires_grad_(True)
    Wd, bd = W.double().cpu(), b.double().cpu()
    proj = [(x @ Wd[k * dp:k * dp + d, :d].t() + bd[k * dp:k * dp + d]) for k in range(3)]
    for t in proj:
        t.retain_grad()
    q = proj[0] / math.sqrt(d)
    s = q @ proj[1].t()
    P = torch.softmax(s, dim=1)
    O = (P * keep / (1.0 - p)) @ proj[2]
    (O * dO[:N, :d].double().cpu()).sum().backward()
    return O.detach(), s.detach(), [t.grad for t in proj], x.grad


def rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).abs().max() / max(1e-30, b.abs().max().item())).item()


@pytest.mark.parametrize("N,d", [(100, 19), (700, 7), (2000, 4), (1300, 32), (257, 13), (300, 10), (150, 23), (64, 1)])
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_small_attention_forward_backward_vs_torch(N, d, p):
    from u2gnn_hip import kernels as K
    Np, dp, X, W, b, dO = _case(N, d, 11 + N + d)
    seed = 0x1234567 + N
    keep = K.dropout_mask(seed, Np, Np, p).double().cpu()[:N, :N] if p > 0 else torch.ones(N, N, dtype=torch.float64)
    O_ref, s_ref, dproj, dx_ref = _ref(X, W, b, dO, N, d, dp, keep, p)
    ws = torch.full((K.attn_small_ws_floats(N, Np, d),), float("nan"), device=DEV)
    O = torch.full((Np, dp), float("nan"), device=DEV)
    ctx = torch.full((K.attn_small_ctx_floats(Np, d),), float("nan"), device=DEV)
    K.attn_small_fwd(X, dp, W, b, dp, d, N, Np, p, seed, O, dp, ctx)
    torch.cuda.synchronize()
    assert rel(O[:N, :d], O_ref) < 2e-5
    assert torch.equal(O[N:], torch.zeros_like(O[N:])) and torch.equal(O[:, d:], torch.zeros_like(O[:, d:]))
    stats = ctx[:2 * Np].view(Np, 2)
    M = s_ref.max(dim=1).values * math.log2(math.e)
    L = torch.exp(s_ref - s_ref.max(dim=1, keepdim=True).values).sum(dim=1)
    assert rel(stats[:N, 0], M) < 1e-5 and rel(stats[:N, 1], 1.0 / L) < 1e-5
    delta = torch.zeros(Np, device=DEV)
    delta[:N] = (O[:N, :d].double() * dO[:N, :d].double()).sum(dim=1).float()
    dQKV = torch.full((Np, 3 * dp), float("nan"), device=DEV)
    dX0 = torch.zeros(Np, dp, device=DEV)
    dX0[:N, :d] = 0.25   # the residual part already there: the kernel adds onto it
    dX = dX0.clone()
    K.attn_small_bwd(ctx, W, dp, d, N, Np, p, seed, dO, dp, delta, 1.0 / math.sqrt(d), dQKV, 3 * dp, dX, dp, ws)
    torch.cuda.synchronize()
    for blk in range(3):
        assert rel(dQKV[:N, blk * dp:blk * dp + d], dproj[blk]) < 2e-5, blk
    pad = dQKV.clone()
    for blk in range(3):
        pad[:N, blk * dp:blk * dp + d] = 0
    assert torch.equal(pad, torch.zeros_like(pad))
    assert rel(dX[:N, :d] - dX0[:N, :d], dx_ref) < 2e-5
    assert torch.equal(dX[N:], dX0[N:]) and torch.equal(dX[:, d:], dX0[:, d:])


def test_small_attention_deterministic_and_guarded():
    from u2gnn_hip import kernels as K
    from u2gnn_hip._lib import U2GNNNativeError
    N, d = 900, 4
    Np, dp, X, W, b, dO = _case(N, d, 5)
    ws = torch.empty(K.attn_small_ws_floats(N, Np, d), device=DEV)
    outs = []
    for _ in range(2):
        O, ctx = torch.empty(Np, dp, device=DEV), torch.empty(K.attn_small_ctx_floats(Np, d), device=DEV)
        K.attn_small_fwd(X, dp, W, b, dp, d, N, Np, 0.5, 7, O, dp, ctx)
        delta = (O * dO).sum(dim=1)
        dQKV, dX = torch.empty(Np, 3 * dp, device=DEV), torch.zeros(Np, dp, device=DEV)
        K.attn_small_bwd(ctx, W, dp, d, N, Np, 0.5, 7, dO, dp, delta, 0.5, dQKV, 3 * dp, dX, dp, ws)
        outs.append((O, ctx, dQKV, dX))
    for a, c in zip(*outs):
        assert torch.equal(a, c)
    # without dX (the first layer of a backward): the same dQKV
    dQKV2 = torch.empty(Np, 3 * dp, device=DEV)
    K.attn_small_bwd(outs[0][1], W, dp, d, N, Np, 0.5, 7, dO, dp, delta, 0.5, dQKV2, 3 * dp, None, dp, ws)
    assert torch.equal(dQKV2, outs[0][2])
    assert K.attn_small_ws_floats(N, Np, 33) < 0 and K.attn_small_ctx_floats(Np, 33) < 0   # d > 32: matrix cores
    with pytest.raises(U2GNNNativeError):
        K.attn_small_fwd(X, dp, W, b, dp, 33, N, Np, 0.5, 7, O, dp, ctx)
    with pytest.raises(U2GNNNativeError):
        K.attn_small_fwd(X, dp, W, b, dp, d, N, Np, 1.0, 7, O, dp, ctx)   # p must be < 1
    with pytest.raises(U2GNNNativeError):   # a context too small for rows_pad
        K.attn_small_fwd(X, dp, W, b, dp, d, N, Np, 0.5, 7, O, dp, ctx[:-4])
    with pytest.raises(U2GNNNativeError):   # a backward scratch too small
        K.attn_small_bwd(ctx, W, dp, d, N, Np, 0.5, 7, dO, dp, delta, 0.5, dQKV, 3 * dp, dX, dp, ws[:-4])
