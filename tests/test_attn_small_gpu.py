"""Small-width node attention (u2gnn_attn_small_fwd / _bwd, csrc/attn_small.hip; d <= 32: the UnSup encoders C3
/ C5 and MUTAG) against a float64 torch restatement of the reference's MHA core on the same dropout masks
(pytorch_U2GNN_UnSup.py:37-40,57: softmax over the N keys, dropout(0.5) on the probabilities with 1/(1-p)
scaling, times V; the backward through torch autograd).  Tolerance 2e-5 of each tensor's scale (the kernels
run exact fp32); padding rows / columns must come out as exact zeros."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(N, d, seed):
    from u2gnn_hip.engine import row_pad
    Np, dp = row_pad(N), 64
    g = torch.Generator(device=DEV).manual_seed(seed)
    QKV = torch.zeros(Np, 3 * dp, device=DEV)
    for b in range(3):
        QKV[:N, b * dp:b * dp + d] = torch.randn(N, d, device=DEV, generator=g) * (1.0 / math.sqrt(d) if b == 0 else 1.0)
    dO = torch.zeros(Np, dp, device=DEV)
    dO[:N, :d] = torch.randn(N, d, device=DEV, generator=g)
    return Np, dp, QKV, dO


def _ref(QKV, dO, N, d, dp, keep, p):
    q = QKV[:N, :d].double().requires_grad_(True)
    k = QKV[:N, dp:dp + d].double().requires_grad_(True)
    v = QKV[:N, 2 * dp:2 * dp + d].double().requires_grad_(True)
    s = q @ k.t()
    P = torch.softmax(s, dim=1)
    Pd = P * keep / (1.0 - p)
    O = Pd @ v
    (O * dO[:N, :d].double()).sum().backward()
    return O.detach(), s.detach(), q.grad, k.grad, v.grad


def rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).abs().max() / max(1e-30, b.abs().max().item())).item()


@pytest.mark.parametrize("N,d", [(100, 19), (700, 7), (2000, 4), (1300, 32), (257, 13), (300, 10), (150, 23), (64, 1)])
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_small_attention_forward_backward_vs_torch(N, d, p):
    from u2gnn_hip import kernels as K
    Np, dp, QKV, dO = _case(N, d, 11 + N + d)
    seed = 0x1234567 + N
    keep = K.dropout_mask(seed, Np, Np, p).double().cpu()[:N, :N] if p > 0 else torch.ones(N, N, dtype=torch.float64)
    O_ref, s_ref, dq, dk, dv = _ref(QKV.cpu(), dO.cpu(), N, d, dp, keep, p)
    ws = torch.full((K.attn_small_ws_floats(N, Np, d),), float("nan"), device=DEV)
    O = torch.full((Np, dp), float("nan"), device=DEV)
    ctx = torch.full((K.attn_small_ctx_floats(Np, d),), float("nan"), device=DEV)
    QKV[N:] = 7.0   # padded rows of the in-projection image hold its bias: they must take no part
    K.attn_small_fwd(QKV, 3 * dp, dp, d, N, Np, p, seed, O, dp, ctx)
    stats = ctx[:2 * Np].view(Np, 2)
    torch.cuda.synchronize()
    assert rel(O[:N, :d], O_ref) < 2e-5
    assert torch.equal(O[N:], torch.zeros_like(O[N:])) and torch.equal(O[:, d:], torch.zeros_like(O[:, d:]))
    M = s_ref.max(dim=1).values * math.log2(math.e)
    L = torch.exp(s_ref - s_ref.max(dim=1, keepdim=True).values).sum(dim=1)
    assert rel(stats[:N, 0], M) < 1e-5 and rel(stats[:N, 1], 1.0 / L) < 1e-5
    delta = torch.zeros(Np, device=DEV)
    delta[:N] = (O[:N, :d].double() * dO[:N, :d].double()).sum(dim=1).float()
    dQKV = torch.full((Np, 3 * dp), float("nan"), device=DEV)
    qs = 0.5
    K.attn_small_bwd(ctx, dp, d, N, Np, p, seed, dO, dp, delta, qs, dQKV, 3 * dp, ws)
    torch.cuda.synchronize()
    assert rel(dQKV[:N, :d], qs * dq) < 2e-5
    assert rel(dQKV[:N, dp:dp + d], dk) < 2e-5
    assert rel(dQKV[:N, 2 * dp:2 * dp + d], dv) < 2e-5
    pad = dQKV.clone()
    pad[:N, :d] = pad[:N, dp:dp + d] = pad[:N, 2 * dp:2 * dp + d] = 0
    assert torch.equal(pad, torch.zeros_like(pad))


def test_small_attention_deterministic_and_guarded():
    from u2gnn_hip import kernels as K
    from u2gnn_hip._lib import U2GNNNativeError
    N, d = 900, 4
    Np, dp, QKV, dO = _case(N, d, 5)
    ws = torch.empty(K.attn_small_ws_floats(N, Np, d), device=DEV)
    outs = []
    for _ in range(2):
        O, ctx = torch.empty(Np, dp, device=DEV), torch.empty(K.attn_small_ctx_floats(Np, d), device=DEV)
        K.attn_small_fwd(QKV, 3 * dp, dp, d, N, Np, 0.5, 7, O, dp, ctx)
        delta = (O * dO).sum(dim=1)
        dQKV = torch.empty(Np, 3 * dp, device=DEV)
        K.attn_small_bwd(ctx, dp, d, N, Np, 0.5, 7, dO, dp, delta, 0.5, dQKV, 3 * dp, ws)
        outs.append((O, ctx, dQKV))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert K.attn_small_ws_floats(N, Np, 33) < 0 and K.attn_small_ctx_floats(Np, 33) < 0   # d > 32: matrix cores
    with pytest.raises(U2GNNNativeError):
        K.attn_small_fwd(QKV, 3 * dp, dp, 33, N, Np, 0.5, 7, O, dp, ctx)
    with pytest.raises(U2GNNNativeError):
        K.attn_small_fwd(QKV, 3 * dp, dp, d, N, Np, 1.0, 7, O, dp, ctx)   # p must be < 1
    with pytest.raises(U2GNNNativeError):   # a context too small for rows_pad
        K.attn_small_fwd(QKV, 3 * dp, dp, d, N, Np, 0.5, 7, O, dp, ctx[:-4])
    with pytest.raises(U2GNNNativeError):   # a backward scratch too small
        K.attn_small_bwd(ctx, dp, d, N, Np, 0.5, 7, dO, dp, delta, 0.5, dQKV, 3 * dp, ws[:-4])
