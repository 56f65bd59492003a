"""Parity of the HIP supervised U2GNN against golden fixtures produced by the REFERENCE
model (tests/golden/make_goldens.py) and against the oracle restatement.

Tolerance (BASELINE.json north_star): max|ours - ref| / max(1, |ref|) <= 1e-3, fp32.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 1e-3


def close(a, b, tol=TOL):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item() <= tol


def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz")))


def _model(z, precision="fp32"):
    from pytorch_U2GNN_Sup import TransformerU2GNN
    bs, k, T, ff, L, d, C, fold = [int(x) for x in z["meta"]]
    m = TransformerU2GNN(feature_dim_size=d, ff_hidden_size=ff, num_classes=C, num_self_att_layers=T, dropout=0.5,
                         num_U2GNN_layers=L, precision=precision)
    sd = {kk[5:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("init.")}
    m.load_state_dict(sd)
    return m.to(DEV), (bs, k, T, ff, L, d, C)


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("name", ["mutag_sup", "mutag_sup_L2T2", "imdbb_sup"])
def test_sup_forward_backward_adam_vs_reference(golden_dir, name, precision):
    from pytorch_U2GNN_Sup import label_smoothing
    from u2gnn_hip.core import DeviceBatch, FusedAdam
    z = _load(golden_dir, name)
    m, (bs, k, T, ff, L, d, C) = _model(z, precision)
    m.eval()
    b = DeviceBatch.from_offsets(z["b0_input_x"], z["b0_offsets"], z["b0_X"], z["b0_labels"])
    # reference-signature path with a sparse graph_pool
    off = z["b0_offsets"]
    B = len(off) - 1
    idx = [[i, j] for i in range(B) for j in range(off[i], off[i + 1])]
    pool = torch.sparse_coo_tensor(torch.tensor(idx).t(), torch.ones(len(idx)), (B, int(off[-1]))).to(DEV)
    scores_ref_sig = m(torch.from_numpy(z["b0_input_x"]).to(DEV), pool, torch.from_numpy(z["b0_X"]).to(DEV))
    assert close(scores_ref_sig.detach(), z["scores"])
    # autograd path: loss.backward() fills p.grad like the reference
    flat = m.flatten_parameters()
    scores = m(b, None, None)
    tgt = label_smoothing(b.labels, C)
    loss = torch.mean(torch.sum(-tgt * torch.log_softmax(scores, 1), 1))
    assert abs(loss.item() - float(z["loss"])) <= TOL * max(1.0, abs(float(z["loss"])))
    for p in m.parameters():
        p.grad = None
    loss.backward()
    for n, p in m.named_parameters():
        assert close(p.grad, z["grad." + n]), n
    # fused clip + Adam on the flat buffers == torch clip_grad_norm_(0.5) + Adam.step()
    for n, p in m.named_parameters():
        flat.grads[n].copy_(p.grad)
    opt = FusedAdam(flat, lr=float(z["lr"]), max_norm=0.5)
    opt.step()
    assert abs(opt.grad_norm() - float(z["grad_norm"])) <= TOL * max(1.0, float(z["grad_norm"]))
    for n, p in m.named_parameters():
        assert close(p.detach(), z["after." + n]), n


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_collab_c4_full_batch_vs_oracle(precision):
    """The benchmark configuration itself (C4: d=367, ff=1024, T=4, k=16, a full 64-graph batch,
    N ~ 4.7K nodes) against the oracle restatement (slot 0, eval mode): scores, loss, grads."""
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.synthetic import collab_like
    np.random.seed(123)
    hb = BatchLoader(collab_like(), 64, 16)()
    torch.manual_seed(123)
    m = TransformerU2GNN(367, 1024, 3, 4, 0.5, 1, precision=precision)
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(DEV).eval()
    flat = m.flatten_parameters()
    b = DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels, device=DEV)
    from u2gnn_hip import kernels as K
    scores, ctx = m.core.forward(b, train=False, need_ctx=True, seed=0)
    dsc = torch.empty_like(scores)
    loss = torch.zeros(1, device=DEV)
    K.smoothed_ce(scores, b.labels, b.B, 3, 0.1, loss, dsc)
    m.core.backward(ctx, dsc, flat.grads)
    torch.set_num_threads(min(16, os.cpu_count()))
    ref = O.sup_forward(sd, torch.from_numpy(hb.input_x), hb.offsets, torch.from_numpy(hb.X_concat), 1, 4,
                        train=False, slots=1)
    lref = O.soft_cross_entropy(ref, O.label_smoothing(torch.from_numpy(hb.labels), 3))
    lref.backward()
    assert close(scores, ref.detach())
    assert abs(loss.item() - lref.item()) <= TOL * max(1.0, abs(lref.item()))
    for n, _ in m.named_parameters():
        assert close(flat.grads[n], sd[n].grad), n


def test_sup_fused_step_matches_autograd(golden_dir):
    """The fused trainer step (kernel CE loss + direct backward into flat grads) equals the
    autograd path."""
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.train import SupTrainer
    z = _load(golden_dir, "imdbb_sup")
    m, (bs, k, T, ff, L, d, C) = _model(z)
    m.eval()
    tr = SupTrainer(m, lr=float(z["lr"]))
    b = DeviceBatch.from_offsets(z["b0_input_x"], z["b0_offsets"], z["b0_X"], z["b0_labels"])
    loss = tr.step(b, train=False)
    assert abs(float(loss) - float(z["loss"])) <= TOL * max(1.0, abs(float(z["loss"])))
    for n, p in m.named_parameters():
        assert close(p.detach(), z["after." + n]), n


def test_train_mode_dropout_matches_oracle_with_kernel_masks(golden_dir):
    """Train mode: the oracle restatement run with the exact masks the kernels draw."""
    from oracle import u2gnn_oracle as O
    from u2gnn_hip import kernels as K
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.engine import SITE_ATTN, SITE_DROP1, SITE_DROP2, SITE_DROPFF, SITE_HEAD, rup, site_seed
    z = _load(golden_dir, "mutag_sup_L2T2")
    m, (bs, k, T, ff, L, d, C) = _model(z)
    m.train()
    b = DeviceBatch.from_offsets(z["b0_input_x"], z["b0_offsets"], z["b0_X"], z["b0_labels"])
    seed = 987654321
    scores, _ = m.core.forward(b, train=True, need_ctx=False, seed=seed)
    N, B = b.N, b.B
    Np, dp = rup(N, 128), rup(d, 64)

    def mk(s, r, c):
        return K.dropout_mask(s, r, c, 0.5).float().cpu()
    masks = {}
    for l in range(L):
        for t in range(T):
            masks[(l, t)] = {"attn": mk(site_seed(seed, l, t, SITE_ATTN), Np, Np)[:N, :N],
                             "drop1": mk(site_seed(seed, l, t, SITE_DROP1), Np, dp)[:N, :d],
                             "drop_ff": mk(site_seed(seed, l, t, SITE_DROPFF), Np, rup(ff, 64))[:N, :ff],
                             "drop2": mk(site_seed(seed, l, t, SITE_DROP2), Np, dp)[:N, :d]}
        masks[("head", l)] = mk(site_seed(seed, l, 0, SITE_HEAD), B, dp)[:, :d]
    sd = {kk: v.detach().cpu() for kk, v in m.state_dict().items()}
    ref = O.sup_forward(sd, torch.from_numpy(z["b0_input_x"]), z["b0_offsets"], torch.from_numpy(z["b0_X"]), L, T,
                        train=True, dropout=0.5, slots=1, masks=masks)
    assert close(scores, ref)
