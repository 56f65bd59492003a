"""Paper-semantics neighbour attention: the window-attention kernels
against a torch fp32 restatement, and the whole supervised model in attention="neighbors" mode
against the oracle (the reference torch encoder fed the transposed window, [k+1, N, d]).  No TF
oracle exists in this image, so this mode's parity is pinned to the restatement only."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import kernels as K  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _ref_window(Q, Kt, V, mask, p):
    """Q, K, V [n, W, dp] (Q pre-scaled); mask [n, W, W] keep decisions."""
    P = torch.softmax(Q @ Kt.transpose(1, 2), dim=-1)
    Pd = P * mask / (1 - p) if p > 0 else P
    return Pd @ V, P


@pytest.mark.parametrize("W,dp,p", [(17, 384, 0.0), (17, 384, 0.5), (5, 64, 0.5), (32, 128, 0.3)])
def test_window_attention_fwd_bwd(W, dp, p):
    n = 37
    rows = n * W
    rows_pad = (rows + 127) // 128 * 128
    g = torch.Generator(device=DEV).manual_seed(1)
    QKV = torch.randn(rows_pad, 3 * dp, device=DEV, generator=g)
    O = torch.full((rows_pad, dp), float("nan"), device=DEV)
    Ps = torch.empty(n, W, W, device=DEV)
    seed = 1234
    K.window_attn_fwd(QKV, W, dp, O, Ps, p, seed, n, rows_pad)
    mask = K.dropout_mask(seed, rows, W, p).float().view(n, W, W) if p > 0 else torch.ones(n, W, W, device=DEV)
    q = QKV[:rows, :dp].view(n, W, dp).clone().requires_grad_(True)
    k = QKV[:rows, dp:2 * dp].view(n, W, dp).clone().requires_grad_(True)
    v = QKV[:rows, 2 * dp:].view(n, W, dp).clone().requires_grad_(True)
    ref, Pref = _ref_window(q, k, v, mask, p)
    assert rel(O[:rows].view(n, W, dp), ref.detach()) < 1e-5
    assert rel(Ps, Pref.detach()) < 1e-5
    assert O[rows:].abs().max().item() == 0 if rows < rows_pad else True
    dO = torch.randn(rows_pad, dp, device=DEV, generator=g)
    dO[rows:] = 0
    ref.backward(dO[:rows].view(n, W, dp))
    dQKV = torch.full((rows_pad, 3 * dp), float("nan"), device=DEV)
    qs = 1 / math.sqrt(7.0)
    K.window_attn_bwd(QKV, W, dp, dO, Ps, p, seed, qs, dQKV, n, rows_pad)
    assert rel(dQKV[:rows, :dp].view(n, W, dp), q.grad * qs) < 1e-5
    assert rel(dQKV[:rows, dp:2 * dp].view(n, W, dp), k.grad) < 1e-5
    assert rel(dQKV[:rows, 2 * dp:].view(n, W, dp), v.grad) < 1e-5
    if rows < rows_pad:
        assert dQKV[rows:].abs().max().item() == 0


def _close(a, b, tol=1e-3):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item() <= tol


@pytest.mark.parametrize("precision,L,T", [("fp32", 1, 2), ("bf16x3", 2, 2), ("fp32", 1, 4)])
def test_sup_neighbors_mode_vs_oracle(golden_dir, precision, L, T):
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.core import DeviceBatch
    z = dict(np.load(os.path.join(golden_dir, "imdbb_sup.npz")))   # real IMDB-BINARY batch (k = 8)
    d, C = int(z["meta"][5]), int(z["meta"][6])
    torch.manual_seed(7)
    m = TransformerU2GNN(d, 256, C, T, 0.5, L, precision=precision, attention="neighbors")
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(DEV).eval()
    flat = m.flatten_parameters()
    b = DeviceBatch.from_offsets(z["b0_input_x"], z["b0_offsets"], z["b0_X"], z["b0_labels"], device=DEV)
    scores, ctx = m.core.forward(b, train=False, need_ctx=True, seed=0)
    dsc = torch.empty_like(scores)
    loss = torch.zeros(1, device=DEV)
    K.smoothed_ce(scores, b.labels, b.B, C, 0.1, loss, dsc)
    m.core.backward(ctx, dsc, flat.grads)
    ref = O.sup_forward(sd, torch.from_numpy(z["b0_input_x"]), z["b0_offsets"], torch.from_numpy(z["b0_X"]), L, T,
                        train=False, attention="neighbors")
    lref = O.soft_cross_entropy(ref, O.label_smoothing(torch.from_numpy(z["b0_labels"]), C))
    lref.backward()
    # fp32 is the parity bar (1e-3).  bf16x3 (the speed mode) gets 5e-3 on gradients: with 9x more
    # tokens per node set, ReLU units sitting at ~0 flip under the split-bf16 rounding (~1e-5) and
    # move single weight-gradient entries by ~2e-3 (measured; fp32 agrees to 1e-4 everywhere)
    gtol = 1e-3 if precision == "fp32" else 5e-3
    assert _close(scores, ref.detach())
    assert abs(loss.item() - lref.item()) <= 1e-3 * max(1.0, abs(lref.item()))
    for n, _ in m.named_parameters():
        assert _close(flat.grads[n], sd[n].grad, gtol), n


def test_sup_neighbors_train_step_runs():
    """Train mode (dropout on, fused trainer) on one batch: finite losses, and the eval-mode loss of
    that batch falls after a few steps."""
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.synthetic import collab_like
    from u2gnn_hip.train import SupTrainer
    np.random.seed(0)
    hb = BatchLoader(collab_like(), 8, 16)()
    torch.manual_seed(0)
    m = TransformerU2GNN(367, 512, 3, 2, 0.5, 1, precision="bf16x3", attention="neighbors").to(DEV).train()
    tr = SupTrainer(m, lr=1e-4, max_norm=0.5, seed=1)
    b = DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels, device=DEV)

    def eval_loss():
        return float(tr.forward_backward(b, train=False).item())
    l0 = eval_loss()
    losses = [float(tr.step(b).item()) for _ in range(10)]
    assert all(np.isfinite(losses))
    assert eval_loss() < l0
