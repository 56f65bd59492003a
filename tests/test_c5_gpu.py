"""C5 (BASELINE configs[4]): U2GNN-UnSup on a REDDIT-MULTI-5K-like batch -- batch 4, k 16, T 4,
ff 1024, d 4, 512 sampled classes, V ~ 2.54 M -- through UnSupTrainer against the oracle
(pytorch_U2GNN_UnSup.py:52-92 composite, sampled_softmax.py:36-56, train_pytorch_U2GNN_UnSup.py:
149-159): per-node logits, loss, every encoder gradient, the ss.weight gradient on the touched rows
(zero elsewhere), and the parameters after one clip(0.5) + Adam step.  Eval mode (no dropout), fixed
sample ids.  Tolerance max|ours - ref| / max(1, |ref|) <= 1e-3 in fp32 and bf16x3."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-3


def close(a, b, tol=TOL):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item() <= tol


@pytest.fixture(scope="module")
def c5_case():
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_UnSup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.synthetic import reddit5k_like
    store = reddit5k_like(seed=0)
    V = int(store.node_start[-1])
    np.random.seed(123)
    hb = BatchLoader(store, 4, 16, with_input_y=True)()
    torch.manual_seed(123)
    m = TransformerU2GNN(feature_dim_size=4, ff_hidden_size=1024, dropout=0.5, num_self_att_layers=4, vocab_size=V,
                         sampled_num=512, num_U2GNN_layers=1, device="cuda")
    sids = m.ss.draw_samples()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    # oracle: loss, dense gradients, one clip + Adam (lr 5e-3: train_pytorch_U2GNN_UnSup.py default)
    names = m.trainable_names()
    prm = {k: sd[k].clone().requires_grad_(True) for k in names}
    enc = {k: v for k, v in prm.items() if k != "ss.weight"}
    logits = O.unsup_forward(enc, prm["ss.weight"], torch.from_numpy(hb.input_x), torch.from_numpy(hb.X_concat),
                             torch.from_numpy(hb.input_y), torch.from_numpy(sids), 1, 4, train=False, slots=1)
    loss = logits.sum()
    loss.backward()
    grads = {k: v.grad.clone() for k, v in prm.items()}
    after = {k: v.detach().clone() for k, v in prm.items()}
    O.clip_and_adam([after[k] for k in names], [grads[k] for k in names], {}, lr=5e-3)
    ref = dict(logits=logits.detach(), loss=float(loss), grads=grads, after=after)
    return m, sd, hb, sids, V, ref


@pytest.mark.parametrize("prec", ["fp32", "bf16x3"])
def test_c5_unsup_trainer_vs_oracle(c5_case, prec):
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.unsup import UnSupTrainer
    m, sd, hb, sids, V, ref = c5_case
    assert V > 2_000_000 and hb.input_x.shape[1] == 17 and 1000 < hb.input_x.shape[0] < 20000
    m.load_state_dict(sd)
    m.precision = prec
    m._core = None
    m = m.to("cuda").eval()
    tr = UnSupTrainer(m, lr=5e-3, max_norm=0.5)
    b = DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, None, device="cuda", input_y=hb.input_y)
    sid = torch.from_numpy(sids).cuda()
    loss = float(tr.forward_backward(b, sid, train=False).item())
    assert close(tr.last_logits, ref["logits"]), "logits"
    assert abs(loss - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"]))
    for n in m.trainable_names():
        if n != "ss.weight":
            assert close(tr.flat.grads[n], ref["grads"][n]), n
    gW, rW = tr.flat.grads["ss.weight"].cpu(), ref["grads"]["ss.weight"]
    rows = np.unique(np.concatenate([hb.input_y, sids]))
    assert close(gW[rows], rW[rows]), "ss.weight gradient rows"
    assert float(gW.abs().sum()) == pytest.approx(float(gW[rows].abs().sum()))   # nothing outside them
    tr.opt.step()
    tr.clear_row_grads()
    assert float(tr.flat.grads["ss.weight"].abs().max()) == 0.0                     # zero between steps
    for n in m.trainable_names():
        assert close(dict(m.named_parameters())[n].detach(), ref["after"][n]), "after." + n


def test_sampled_softmax_rows_equal_dense_backward():
    """ABI v9 compact rows folded by index_add_rows == the dense atomics backward, bit for bit
    (two addends per element at most, onto zero), including labels that are also samples."""
    from u2gnn_hip import kernels as K
    g = torch.Generator(device="cuda").manual_seed(5)
    V, D, N, S = 5000, 12, 300, 128
    W = torch.randn(V, D, device="cuda", generator=g)
    X = torch.randn(N, D, device="cuda", generator=g)
    labels = torch.randperm(V, device="cuda", generator=g)[:N]
    sids = torch.cat([labels[:40], torch.randperm(V, device="cuda", generator=g)[:S - 40]])
    sids = torch.unique(sids)[:S]
    S = sids.numel()
    loss, prob = torch.empty(N, device="cuda"), torch.empty(N, S, device="cuda")
    K.sampled_softmax_fwd(X, D, labels, sids, S, W, D, loss, prob, N, D)
    dX0, dW0 = torch.empty_like(X), torch.zeros_like(W)
    K.sampled_softmax_bwd(X, D, labels, sids, S, W, D, prob, None, dX0, D, dW0, D, N, D)
    dX1, dW1 = torch.empty_like(X), torch.zeros_like(W)
    rl, rs = torch.empty(N, D, device="cuda"), torch.empty(S, D, device="cuda")
    K.sampled_softmax_bwd_rows(X, D, labels, sids, S, W, D, prob, None, dX1, D, rl, rs, N, D)
    K.index_add_rows(rl, labels, dW1)
    K.index_add_rows(rs, sids, dW1)
    assert torch.equal(dX0, dX1)
    assert torch.equal(dW0, dW1)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    K.index_zero_rows(torch.cat([labels, sids]), dW1, err)
    assert float(dW1.abs().max()) == 0.0 and int(err.item()) == 0
    K.index_add_rows(rl[:2], torch.tensor([0, V], device="cuda"), dW1, 0.5, err)   # V is out of range
    assert int(err.item()) == 1 and torch.equal(dW1[0], 0.5 * rl[0])
