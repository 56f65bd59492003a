"""The forward tail of a mid-width encoder layer (u2gnn_layer_tail_mid_fwd, csrc/mid_layer.hip; 32 < d <= 256 with a
few hundred rows: C2's IMDBBINARY batches) against a float64 torch restatement of the reference's
TransformerEncoderLayer tail on the kernels' own dropout masks (pytorch_U2GNN_Sup.py:19-21,35: out_proj -> dropout ->
+ x -> norm1 -> linear1 -> ReLU -> dropout -> linear2 -> dropout -> + x -> norm2, post-LN, eps 1e-5).  Exact fp32 on
the vector ALUs: 1e-4 of each tensor's scale; padding rows / columns exact zeros; two runs give the same bits."""
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


def _case(N, d, ff, p):
    from u2gnn_hip import kernels as K
    from u2gnn_hip.engine import row_pad
    Np, dp, ffp = row_pad(N), -(-d // 64) * 64, -(-ff // 64) * 64
    g = torch.Generator(device="cpu").manual_seed(N + d + ff)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)   # noqa: E731
    Wo, bo, W1, b1, W2, b2 = r(d, d) / d ** 0.5, r(d) * 0.1, r(ff, d) / d ** 0.5, r(ff) * 0.1, r(d, ff) / ff ** 0.5, r(d) * 0.1
    n1w, n1b, n2w, n2b = 1 + 0.1 * r(d), 0.1 * r(d), 1 + 0.1 * r(d), 0.1 * r(d)
    O, X = r(N, d), r(N, d)
    seeds = (0x4444 + N, 0x5555 + d, 0x6666 + ff)
    f32 = lambda t, rows, cols: torch.nn.functional.pad(t, (0, cols - t.shape[1], 0, rows - t.shape[0])).float().to(DEV)  # noqa: E731
    pad1 = lambda t, n: torch.nn.functional.pad(t, (0, n - t.shape[0])).float().to(DEV)   # noqa: E731
    w = dict(W_o=f32(Wo, dp, dp), b_o=pad1(bo, dp), n1_w=n1w.float().to(DEV), n1_b=n1b.float().to(DEV),
             W1=f32(W1, ffp, dp), b1=pad1(b1, ffp), W2=f32(W2, dp, ffp), b2=pad1(b2, dp), n2_w=n2w.float().to(DEV),
             n2_b=n2b.float().to(DEV))
    nan = lambda *s: torch.full(s, float("nan"), device=DEV)   # noqa: E731
    fw = dict(O=f32(O, Np, dp), X=f32(X, Np, dp), Z1=nan(Np, dp), X1=nan(Np, dp), mean1=nan(Np), rstd1=nan(Np),
              Hd=nan(Np, ffp), Z2=nan(Np, dp), X2=nan(Np, dp), mean2=nan(Np), rstd2=nan(Np))
    ws = torch.full((K.layer_tail_mid_ws_floats(Np, dp, ffp),), float("nan"), device=DEV)
    K.layer_tail_mid_fwd(N, Np, d, dp, ff, ffp, p, seeds, ws, **w, **fw)
    torch.cuda.synchronize()
    return K, Np, dp, ffp, seeds, (Wo, bo, W1, b1, W2, b2, n1w, n1b, n2w, n2b, O, X), w, fw, ws


@pytest.mark.parametrize("N,d,ff", [(80, 136, 1024), (100, 100, 256), (300, 67, 128), (500, 256, 200), (8, 33, 64),
                                    (130, 64, 1024)])
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_mid_tail_forward_vs_torch(N, d, ff, p):
    K, Np, dp, ffp, seeds, ref_in, w, fw, ws = _case(N, d, ff, p)
    Wo, bo, W1, b1, W2, b2, n1w, n1b, n2w, n2b, O, X = ref_in
    m = [K.dropout_mask(s, Np, c, p).double().cpu() if p > 0 else torch.ones(Np, c, dtype=torch.float64)
         for s, c in zip(seeds, (dp, ffp, dp))]
    m1, mff, m2 = m[0][:N, :d], m[1][:N, :ff], m[2][:N, :d]
    z1 = m1 * (O @ Wo.t() + bo) / (1 - p) + X
    x1, mu1, rs1 = _ln(z1, n1w, n1b)
    h = mff * torch.relu(x1 @ W1.t() + b1) / (1 - p)
    z2 = m2 * (h @ W2.t() + b2) / (1 - p) + x1
    x2, mu2, rs2 = _ln(z2, n2w, n2b)
    for k, ref in dict(Z1=z1, X1=x1, Hd=h, Z2=z2, X2=x2).items():
        t = fw[k]
        assert rel(t[:N, :ref.shape[1]], ref) < 1e-4, k
        pad = t.clone()
        pad[:N, :ref.shape[1]] = 0
        assert torch.equal(pad, torch.zeros_like(pad)), f"{k}: padding not zero"
    for k, ref in (("mean1", mu1), ("rstd1", rs1), ("mean2", mu2), ("rstd2", rs2)):
        assert rel(fw[k][:N], ref) < 1e-4, k
        assert torch.equal(fw[k][N:], torch.zeros_like(fw[k][N:])), k


def test_mid_tail_deterministic():
    a = _case(300, 136, 1024, 0.5)[7]
    b = _case(300, 136, 1024, 0.5)[7]
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_mid_tail_guards():
    from u2gnn_hip import kernels as K
    from u2gnn_hip._lib import U2GNNNativeError
    assert K.layer_tail_mid_ws_floats(128, 320, 1024) == -1   # dp > 256
    N, Np, d, dp, ff, ffp = 10, 128, 300, 320, 64, 64
    t = {k: torch.zeros(Np, max(dp, ffp), device=DEV) for k in ("W_o", "b_o", "n1_w", "n1_b", "W1", "b1", "W2", "b2",
                                                                 "n2_w", "n2_b", "O", "X", "Z1", "X1", "mean1", "rstd1",
                                                                 "Hd", "Z2", "X2", "mean2", "rstd2")}
    with pytest.raises(U2GNNNativeError):
        K.layer_tail_mid_fwd(N, Np, d, dp, ff, ffp, 0.5, (1, 2, 3), torch.zeros(1 << 20, device=DEV), **t)
