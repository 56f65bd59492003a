"""A whole small-width encoder layer (u2gnn_layer_small_fwd / _bwd, csrc/small_layer.hip; d <= 32) -- in-projection,
node attention with dropout, out-projection, LayerNorm1, FFN, LayerNorm2 and the full backward -- against a float64
torch restatement of torch.nn.TransformerEncoderLayer(d, nhead=1, ff, dropout=p), post-LN
(pytorch_U2GNN_UnSup.py:37-40,57), on the kernels' own dropout masks.  Row counts on both sides of the fusion
threshold (rows_pad >= 1024: attention + tail and tail backward + dQ walk each in one launch; below: separate
launches).  Exact fp32 kernels: 1e-4 of each tensor's scale; padding rows / columns exact zeros."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / max(1e-30, b.abs().max().item())).item()


def _ln(z, w, b):
    mu = z.mean(dim=1, keepdim=True)
    var = ((z - mu) ** 2).mean(dim=1, keepdim=True)
    return (z - mu) / torch.sqrt(var + 1e-5) * w + b


@pytest.mark.parametrize("N,d,ff", [(1914, 4, 1024), (1100, 19, 256), (700, 7, 1024), (1030, 32, 128)])
@pytest.mark.parametrize("p", [0.0, 0.5])
@pytest.mark.parametrize("need_dx", [True, False])
def test_small_layer_vs_torch(N, d, ff, p, need_dx):
    from u2gnn_hip import kernels as K
    from u2gnn_hip.engine import row_pad
    Np, dp, ffp = row_pad(N), 64, -(-ff // 64) * 64
    g = torch.Generator(device="cpu").manual_seed(N + 3 * d + ff)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)   # noqa: E731
    Win, bin_ = r(3 * d, d) / d ** 0.5, 0.1 * r(3 * d)
    Wo, bo, W1, b1, W2, b2 = r(d, d) / d ** 0.5, r(d) * 0.1, r(ff, d) / d ** 0.5, r(ff) * 0.1, r(d, ff) / ff ** 0.5, r(d) * 0.1
    n1w, n1b, n2w, n2b = 1 + 0.1 * r(d), 0.1 * r(d), 1 + 0.1 * r(d), 0.1 * r(d)
    X, dX2 = r(N, d), r(N, d)
    seeds, sa = (0x51 + N, 0x52 + d, 0x53 + ff), 0x54 + N
    mk = lambda s, c: (K.dropout_mask(s, Np, c, p).double().cpu() if p > 0   # noqa: E731
                       else torch.ones(Np, c, dtype=torch.float64))
    mA, m1, mff, m2 = mk(sa, Np)[:N, :N], mk(seeds[0], dp)[:N, :d], mk(seeds[1], ffp)[:N, :ff], mk(seeds[2], dp)[:N, :d]
    # float64 reference with autograd on every intermediate the kernels write
    Xt = X.clone().requires_grad_(True)
    proj = [Xt @ Win[k * d:(k + 1) * d].t() + bin_[k * d:(k + 1) * d] for k in range(3)]
    for t in proj:
        t.retain_grad()
    P = torch.softmax((proj[0] / math.sqrt(d)) @ proj[1].t(), dim=1)
    O = (P * mA / (1 - p)) @ proj[2]
    O.retain_grad()
    A = O @ Wo.t() + bo
    A.retain_grad()
    x1 = _ln(m1 * A / (1 - p) + Xt, n1w, n1b)
    x1.retain_grad()
    a = x1 @ W1.t() + b1
    a.retain_grad()
    h = mff * torch.relu(a) / (1 - p)
    F = h @ W2.t() + b2
    F.retain_grad()
    x2 = _ln(m2 * F / (1 - p) + x1, n2w, n2b)
    (x2 * dX2).sum().backward()

    f32 = lambda t, rows, cols: torch.nn.functional.pad(t, (0, cols - t.shape[1], 0, rows - t.shape[0])).float().to(DEV)  # noqa: E731
    pad1 = lambda t, n: torch.nn.functional.pad(t, (0, n - t.shape[0])).float().to(DEV)   # noqa: E731
    W_in = torch.zeros(3 * dp, dp, device=DEV)
    b_in = torch.zeros(3 * dp, device=DEV)
    for k in range(3):
        W_in[k * dp:k * dp + d, :d] = Win[k * d:(k + 1) * d].float().to(DEV)
        b_in[k * dp:k * dp + d] = bin_[k * d:(k + 1) * d].float().to(DEV)
    w = dict(W_o=f32(Wo, dp, dp), b_o=pad1(bo, dp), n1_w=n1w.float().to(DEV), n1_b=n1b.float().to(DEV),
             W1=f32(W1, ffp, dp), b1=pad1(b1, ffp), W2=f32(W2, dp, ffp), b2=pad1(b2, dp), n2_w=n2w.float().to(DEV),
             n2_b=n2b.float().to(DEV))
    nan = lambda *s: torch.full(s, float("nan"), device=DEV)   # noqa: E731
    fw = dict(O=nan(Np, dp), X=f32(X, Np, dp), Z1=nan(Np, dp), X1=nan(Np, dp), mean1=nan(Np), rstd1=nan(Np),
              Hd=nan(Np, ffp), Z2=nan(Np, dp), X2=nan(Np, dp), mean2=nan(Np), rstd2=nan(Np))
    ctx = torch.full((K.attn_small_ctx_floats(Np, d),), float("nan"), device=DEV)
    K.layer_small_fwd(N, Np, d, dp, ff, ffp, p, seeds, sa, W_in, b_in, ctx, **w, **fw)
    torch.cuda.synchronize()
    for k, ref in dict(O=O, X1=x1, Hd=h, X2=x2).items():
        t = fw[k]
        assert rel(t[:N, :ref.shape[1]], ref.detach()) < 1e-4, k
        pad = t.clone()
        pad[:N, :ref.shape[1]] = 0
        assert torch.equal(pad, torch.zeros_like(pad)), f"{k}: padding not zero"
    bw = dict(dX2=f32(dX2, Np, dp), dX1=nan(Np, dp), dF=nan(Np, dp), dH=nan(Np, ffp), dX=nan(Np, dp), dA=nan(Np, dp),
              dO=nan(Np, dp), delta=nan(Np))
    dQKV = torch.full((Np, 3 * dp), float("nan"), device=DEV)
    ws = torch.full((K.attn_small_ws_floats(N, Np, d),), float("nan"), device=DEV)
    fw_in = {k: v for k, v in fw.items() if k != "X2"}
    K.layer_small_bwd(N, Np, d, dp, ff, ffp, p, seeds, sa, W_in, ctx, dQKV, need_dx, ws, **w, **fw_in, **bw)
    torch.cuda.synchronize()
    for k, ref in dict(dX1=x1.grad, dF=F.grad, dH=a.grad, dA=A.grad, dO=O.grad).items():
        assert rel(bw[k][:N, :ref.shape[1]], ref) < 1e-4, k
    for blk in range(3):
        assert rel(dQKV[:N, blk * dp:blk * dp + d], proj[blk].grad) < 1e-4, blk
    pad = dQKV.clone()
    for blk in range(3):
        pad[:N, blk * dp:blk * dp + d] = 0
    assert torch.equal(pad, torch.zeros_like(pad))
    assert rel(bw["delta"][:N], (O.grad * O.detach()).sum(dim=1)) < 1e-4
    if need_dx:   # the residual branch plus the in-projection's dQKV W_in
        assert rel(bw["dX"][:N, :d], Xt.grad) < 1e-4
    assert torch.equal(bw["dX"][N:], torch.zeros_like(bw["dX"][N:]))


def test_small_layer_deterministic():
    """Two runs of the fused forms give the same bits (fixed partitions and merge orders)."""
    from u2gnn_hip import kernels as K
    from u2gnn_hip.engine import row_pad
    N, d, ff = 1500, 4, 1024
    Np, dp, ffp = row_pad(N), 64, 1024
    gen = torch.Generator(device=DEV).manual_seed(3)
    rn = lambda *s: torch.randn(*s, device=DEV, generator=gen)   # noqa: E731
    W_in, b_in = torch.zeros(3 * dp, dp, device=DEV), torch.zeros(3 * dp, device=DEV)
    for k in range(3):
        W_in[k * dp:k * dp + d, :d] = rn(d, d) * 0.5
    w = dict(W_o=torch.zeros(dp, dp, device=DEV), b_o=torch.zeros(dp, device=DEV), n1_w=torch.ones(d, device=DEV),
             n1_b=torch.zeros(d, device=DEV), W1=torch.zeros(ffp, dp, device=DEV), b1=0.1 * rn(ffp),
             W2=torch.zeros(dp, ffp, device=DEV), b2=torch.zeros(dp, device=DEV), n2_w=torch.ones(d, device=DEV),
             n2_b=torch.zeros(d, device=DEV))
    w["W_o"][:d, :d] = rn(d, d)
    w["W1"][:, :d] = rn(ffp, d)
    w["W2"][:d, :] = rn(d, ffp) * 0.05
    X = torch.zeros(Np, dp, device=DEV)
    X[:N, :d] = rn(N, d)
    outs = []
    for _ in range(2):
        fw = {k: torch.empty(Np, c, device=DEV) for k, c in (("O", dp), ("Z1", dp), ("X1", dp), ("Hd", ffp), ("Z2", dp),
                                                                ("X2", dp))}
        fw.update({k: torch.empty(Np, device=DEV) for k in ("mean1", "rstd1", "mean2", "rstd2")})
        ctx = torch.empty(K.attn_small_ctx_floats(Np, d), device=DEV)
        K.layer_small_fwd(N, Np, d, dp, ff, ffp, 0.5, (1, 2, 3), 4, W_in, b_in, ctx, X=X, **w, **fw)
        bw = {k: torch.empty(Np, c, device=DEV) for k, c in (("dX1", dp), ("dF", dp), ("dH", ffp), ("dX", dp),
                                                                ("dA", dp), ("dO", dp))}
        bw["delta"] = torch.empty(Np, device=DEV)
        dQKV = torch.empty(Np, 3 * dp, device=DEV)
        ws = torch.empty(K.attn_small_ws_floats(N, Np, d), device=DEV)
        fw_in = {k: v for k, v in fw.items() if k != "X2"}
        K.layer_small_bwd(N, Np, d, dp, ff, ffp, 0.5, (1, 2, 3), 4, W_in, ctx, dQKV, True, ws, dX2=fw["X2"], X=X,
                          **w, **fw_in, **bw)
        outs.append([fw[k] for k in sorted(fw)] + [bw[k] for k in sorted(bw)] + [dQKV, ctx])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
