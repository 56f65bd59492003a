"""The row-local tail of a small-width encoder layer (u2gnn_layer_tail_small_fwd / _bwd, csrc/small_layer.hip; d <= 32:
the UnSup encoders C3 / C5 and MUTAG) against a float64 torch restatement of the reference's TransformerEncoderLayer
tail on the kernels' own dropout masks (pytorch_U2GNN_UnSup.py:37-40,57: out_proj -> dropout -> + x -> norm1 ->
linear1 -> ReLU -> dropout -> linear2 -> dropout -> + x -> norm2, post-LN, eps 1e-5), the backward through torch
autograd.  The kernels run exact fp32: tolerance 1e-4 of each tensor's scale (LayerNorm's backward divides by
the row's standard deviation); padding rows / columns must come out as exact zeros."""
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
    return (z - mu) / torch.sqrt(var + 1e-5) * w + b, mu.squeeze(1), 1.0 / torch.sqrt(var.squeeze(1) + 1e-5)


@pytest.mark.parametrize("N,d,ff", [(1914, 4, 1024), (100, 19, 1024), (300, 7, 256), (77, 32, 100), (8, 1, 64)])
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_small_tail_forward_backward_vs_torch(N, d, ff, p):
    from u2gnn_hip import kernels as K
    from u2gnn_hip.engine import row_pad
    Np, dp, ffp = row_pad(N), 64, -(-ff // 64) * 64
    g = torch.Generator(device="cpu").manual_seed(N + d + ff)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)   # noqa: E731
    Wo, bo, W1, b1, W2, b2 = r(d, d) / d ** 0.5, r(d) * 0.1, r(ff, d) / d ** 0.5, r(ff) * 0.1, r(d, ff) / ff ** 0.5, r(d) * 0.1
    n1w, n1b, n2w, n2b = 1 + 0.1 * r(d), 0.1 * r(d), 1 + 0.1 * r(d), 0.1 * r(d)
    O, X, dX2 = r(N, d), r(N, d), r(N, d)
    seeds = (0x1111 + N, 0x2222 + d, 0x3333 + ff)
    m = [K.dropout_mask(s, Np, c, p).double().cpu() if p > 0 else torch.ones(Np, c, dtype=torch.float64)
         for s, c in zip(seeds, (dp, ffp, dp))]
    m1, mff, m2 = m[0][:N, :d], m[1][:N, :ff], m[2][:N, :d]
    # float64 reference with autograd on every intermediate the kernels write
    Ot, Xt = O.clone().requires_grad_(True), X.clone().requires_grad_(True)
    A = Ot @ Wo.t() + bo
    A.retain_grad()
    z1 = m1 * A / (1 - p) + Xt
    x1, mu1, rs1 = _ln(z1, n1w, n1b)
    x1.retain_grad()
    a = x1 @ W1.t() + b1
    a.retain_grad()
    h = mff * torch.relu(a) / (1 - p)
    F = h @ W2.t() + b2
    F.retain_grad()
    z2 = m2 * F / (1 - p) + x1
    x2, mu2, rs2 = _ln(z2, n2w, n2b)
    (x2 * dX2).sum().backward()

    f32 = lambda t, rows, cols: torch.nn.functional.pad(t, (0, cols - t.shape[1], 0, rows - t.shape[0])).float().to(DEV)  # noqa: E731
    pad1 = lambda t, n: torch.nn.functional.pad(t, (0, n - t.shape[0])).float().to(DEV)   # noqa: E731
    w = dict(W_o=f32(Wo, dp, dp), b_o=pad1(bo, dp), n1_w=n1w.float().to(DEV), n1_b=n1b.float().to(DEV),
             W1=f32(W1, ffp, dp), b1=pad1(b1, ffp), W2=f32(W2, dp, ffp), b2=pad1(b2, dp), n2_w=n2w.float().to(DEV),
             n2_b=n2b.float().to(DEV))
    nan = lambda *s: torch.full(s, float("nan"), device=DEV)   # noqa: E731
    fw = dict(O=f32(O, Np, dp), X=f32(X, Np, dp), Z1=nan(Np, dp), X1=nan(Np, dp), mean1=nan(Np), rstd1=nan(Np),
              Hd=nan(Np, ffp), Z2=nan(Np, dp), X2=nan(Np, dp), mean2=nan(Np), rstd2=nan(Np))
    K.layer_tail_small(False, N, Np, d, dp, ff, ffp, p, seeds, **w, **fw)
    torch.cuda.synchronize()
    exp = dict(Z1=z1, X1=x1, Hd=h, Z2=z2, X2=x2)
    for k, ref in exp.items():
        t = fw[k]
        assert rel(t[:N, :ref.shape[1]], ref.detach()) < 1e-4, k
        pad = t.clone()
        pad[:N, :ref.shape[1]] = 0
        assert torch.equal(pad, torch.zeros_like(pad)), f"{k}: padding not zero"
    for k, ref in (("mean1", mu1), ("rstd1", rs1), ("mean2", mu2), ("rstd2", rs2)):
        assert rel(fw[k][:N], ref.detach()) < 1e-4, k
        assert torch.equal(fw[k][N:], torch.zeros_like(fw[k][N:])), k
    bw = dict(dX2=f32(dX2, Np, dp), dX1=nan(Np, dp), dF=nan(Np, dp), dH=nan(Np, ffp), dX=nan(Np, dp), dA=nan(Np, dp),
              dO=nan(Np, dp), delta=nan(Np))
    fw_in = {k: v for k, v in fw.items() if k != "X2"}
    K.layer_tail_small(True, N, Np, d, dp, ff, ffp, p, seeds, **w, **fw_in, **bw)
    torch.cuda.synchronize()
    exp = dict(dX1=x1.grad, dF=F.grad, dH=a.grad, dX=Xt.grad, dA=A.grad, dO=Ot.grad)
    for k, ref in exp.items():
        t = bw[k]
        assert rel(t[:N, :ref.shape[1]], ref) < 1e-4, k
        pad = t.clone()
        pad[:N, :ref.shape[1]] = 0
        assert torch.equal(pad, torch.zeros_like(pad)), f"{k}: padding not zero"
    delta = (Ot.grad * O).sum(dim=1)
    assert rel(bw["delta"][:N], delta) < 1e-4
    assert torch.equal(bw["delta"][N:], torch.zeros_like(bw["delta"][N:]))


def test_small_tail_guards():
    from u2gnn_hip import kernels as K
    from u2gnn_hip._lib import U2GNNNativeError
    N, Np, d, dp, ff, ffp = 10, 128, 40, 64, 64, 64   # d > 32: the matrix-core path's
    t = {k: torch.zeros(Np, max(dp, ffp), device=DEV) for k in ("W_o", "b_o", "n1_w", "n1_b", "W1", "b1", "W2", "b2",
                                                                 "n2_w", "n2_b", "O", "X", "Z1", "X1", "mean1", "rstd1",
                                                                 "Hd", "Z2", "X2", "mean2", "rstd2")}
    with pytest.raises(U2GNNNativeError):
        K.layer_tail_small(False, N, Np, d, dp, ff, ffp, 0.5, (1, 2, 3), **t)
    with pytest.raises(U2GNNNativeError):   # the backward needs its gradient buffers
        K.layer_tail_small(True, N, Np, 4, dp, ff, ffp, 0.5, (1, 2, 3), **t)
