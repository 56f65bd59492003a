"""Generate the golden fixtures in tests/golden/ (run in the survey/build container only).

Sources of truth:
  * the REFERENCE model ``pytorch_U2GNN_Sup.TransformerU2GNN`` imported from
    /root/reference/U2GNN_pytorch (its only import is torch),
  * the REFERENCE ``sampled_softmax.SampledSoftmax`` with the REFERENCE C++/Cython
    log-uniform sampler compiled from /root/reference sources by
    oracle/build_ref_sampler.sh into oracle/_ref/,
  * batches from oracle.u2gnn_oracle (sequential restatement of get_batch_data with the
    seed-123 numpy stream; the reference's util.py cannot be imported — it needs pyriemann).

The fixtures are data only (inputs + expected outputs).  Nothing of the reference's
source is stored.  Usage:  python tests/golden/make_goldens.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference/U2GNN_pytorch"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle", "_ref"))
sys.path.insert(0, REF)

from oracle import u2gnn_oracle as O  # noqa: E402

import pytorch_U2GNN_Sup as REF_SUP  # noqa: E402  (reference model, torch-only import)
from sampled_softmax import SampledSoftmax as REF_SS  # noqa: E402
from log_uniform import LogUniformSampler as REF_LUS  # noqa: E402


def _sd_np(model):
    return {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}


def sup_case(name, dataset, deg_tag, bs, k, T, ff, L, lr=0.0005, n_batches=3, fold=1):
    graphs, C = O.load_data(os.path.join(REPO, "dataset", dataset, dataset + ".txt"), deg_tag)
    labels = [g.label for g in graphs]
    tr, te = O.separate_data_idx(labels, fold)
    train_graphs = [graphs[i] for i in tr]
    d = graphs[0].node_features.shape[1]
    np.random.seed(123)
    torch.manual_seed(123)
    batches = []
    for _ in range(n_batches):
        sel = np.random.permutation(len(train_graphs))[:bs]
        bg = [train_graphs[i] for i in sel]
        batches.append((sel,) + O.get_batch_data_seq(bg, k))
    model = REF_SUP.TransformerU2GNN(feature_dim_size=d, ff_hidden_size=ff, num_classes=C,
                                     dropout=0.5, num_self_att_layers=T, num_U2GNN_layers=L)
    sd0 = _sd_np(model)
    out = {"meta": np.array([bs, k, T, ff, L, d, C, fold], np.int64), "lr": np.float32(lr),
           "train_idx": np.asarray(tr, np.int64), "test_idx": np.asarray(te, np.int64)}
    for i, (sel, ix, off, X, y) in enumerate(batches):
        out[f"b{i}_sel"] = sel.astype(np.int64)
        out[f"b{i}_input_x"] = ix
        out[f"b{i}_offsets"] = off
        out[f"b{i}_labels"] = y
        out[f"b{i}_X"] = X
    # batch 0: eval-mode forward, loss, grads, one clip+Adam step (reference modules)
    sel, ix, off, X, y = batches[0]
    Nn = int(off[-1])
    B = len(off) - 1
    idx = [[b, j] for b in range(B) for j in range(off[b], off[b + 1])]
    pool = torch.sparse_coo_tensor(torch.LongTensor(idx).t(), torch.ones(Nn), (B, Nn))
    model.eval()
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    opt.zero_grad()
    scores = model(torch.from_numpy(ix), pool, torch.from_numpy(X))
    tgt = REF_SUP.label_smoothing(torch.from_numpy(y), C)
    loss = torch.mean(torch.sum(-tgt * torch.log_softmax(scores, 1), 1))
    loss.backward()
    out["scores"] = scores.detach().numpy()
    out["loss"] = np.float32(loss.item())
    for k_, p in model.named_parameters():
        out["grad." + k_] = p.grad.numpy().copy()
    total = torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
    out["grad_norm"] = np.float32(total.item())
    opt.step()
    for k_, v in sd0.items():
        out["init." + k_] = v
    for k_, p in model.named_parameters():
        out["after." + k_] = p.detach().numpy().copy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    # pin the oracle restatement against the reference on this case
    sd = {k_: torch.from_numpy(v) for k_, v in sd0.items()}
    s2 = O.sup_forward(sd, torch.from_numpy(ix), off, torch.from_numpy(X), L, T, train=False)
    err = (s2 - torch.from_numpy(out["scores"])).abs().max().item()
    print(f"{name}: N={Nn} d={d} C={C} loss={out['loss']:.6f} oracle|d|={err:.2e}")
    assert err < 1e-4


def sampler_case():
    out = {}
    for V in (8792, 2542091):
        s = REF_LUS(V)
        for c in range(3):
            ids, tf, sf = s.sample(512, np.arange(4, dtype=np.int64))
            out[f"V{V}_c{c}_ids_order"] = np.asarray(ids, np.int64)   # unordered_set order
            out[f"V{V}_c{c}_sample_freq"] = np.asarray(sf, np.float32)
            out[f"V{V}_c{c}_true_freq"] = np.asarray(tf, np.float32)
    np.savez_compressed(os.path.join(HERE, "sampler.npz"), **out)
    print("sampler fixtures written")


def sampled_softmax_case():
    torch.manual_seed(7)
    V, D, Nn = 8792, 19, 102
    ss = REF_SS(V, 512, D, "cpu")
    x = torch.randn(Nn, D, requires_grad=True)
    labels = torch.arange(300, 300 + Nn, dtype=torch.long)
    sv = REF_LUS(V).sample(512, labels.numpy())
    logits = ss.sampled(x, labels, sv)
    logits.sum().backward()
    np.savez_compressed(os.path.join(HERE, "sampled_softmax.npz"),
                        weight=ss.weight.detach().numpy(), inputs=x.detach().numpy(),
                        labels=labels.numpy(), sample_ids=np.asarray(sv[0], np.int64),
                        logits=logits.detach().numpy(), grad_inputs=x.grad.numpy(),
                        grad_weight=ss.weight.grad.numpy())
    print("sampled softmax fixture written")


def unsup_case(name="ptc_unsup", dataset="PTC", bs=4, k=4, T=2, ff=1024, L=1, lr=0.005):
    """C3: reference encoder stack (Sup class's u2gnn_layers, identical TransformerEncoder
    construction) + reference SampledSoftmax, glued per SURVEY §8 a12; eval mode."""
    graphs, _ = O.load_data(os.path.join(REPO, "dataset", dataset, dataset + ".txt"), False)
    d = graphs[0].node_features.shape[1]
    starts = np.cumsum([0] + [g.n for g in graphs])
    V = int(starts[-1])
    np.random.seed(123)
    torch.manual_seed(123)
    sel = np.random.permutation(len(graphs))[:bs]
    ix, off, X, _ = O.get_batch_data_seq([graphs[i] for i in sel], k)
    iy = np.concatenate([np.arange(starts[i], starts[i + 1]) for i in sel]).astype(np.int64)
    enc = REF_SUP.TransformerU2GNN(feature_dim_size=d, ff_hidden_size=ff, num_classes=2,
                                   dropout=0.5, num_self_att_layers=T, num_U2GNN_layers=L)
    ss = REF_SS(V, 512, d * L, "cpu")
    sv = REF_LUS(V).sample(512, iy)
    enc.eval()
    params = list(enc.u2gnn_layers.parameters()) + [ss.weight]
    opt = torch.optim.Adam(params, lr=lr)
    inp = torch.nn.functional.embedding(torch.from_numpy(ix), torch.from_numpy(X))
    outs = []
    for l in range(L):
        o = enc.u2gnn_layers[l](inp)[:, 0, :]
        outs.append(o)
        inp = torch.nn.functional.embedding(torch.from_numpy(ix), o)
    ov = torch.cat(outs, 1)
    logits = ss.sampled(ov, torch.from_numpy(iy), sv)
    loss = logits.sum()
    loss.backward()
    out = {"meta": np.array([bs, k, T, ff, L, d, V], np.int64), "lr": np.float32(lr),
           "sel": sel.astype(np.int64), "input_x": ix, "offsets": off, "input_y": iy, "X": X,
           "sample_ids": np.asarray(sv[0], np.int64), "logits": logits.detach().numpy(),
           "loss": np.float32(loss.item())}
    sd0 = {}
    for kk, p in enc.u2gnn_layers.named_parameters():
        out["grad.u2gnn_layers." + kk] = p.grad.numpy().copy()
    out["grad.ss.weight"] = ss.weight.grad.numpy().copy()
    # initial params were overwritten by nothing yet (grads only): record them now
    for kk, p in enc.u2gnn_layers.named_parameters():
        out["init.u2gnn_layers." + kk] = p.detach().numpy().copy()
        sd0["u2gnn_layers." + kk] = p.detach().clone()
    out["init.ss.weight"] = ss.weight.detach().numpy().copy()
    w0 = ss.weight.detach().clone()
    total = torch.nn.utils.clip_grad_norm_(params, 0.5)
    out["grad_norm"] = np.float32(total.item())
    opt.step()
    for kk, p in enc.u2gnn_layers.named_parameters():
        out["after.u2gnn_layers." + kk] = p.detach().numpy().copy()
    out["after.ss.weight"] = ss.weight.detach().numpy().copy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    lg = O.unsup_forward(sd0, w0, torch.from_numpy(ix), torch.from_numpy(X), torch.from_numpy(iy),
                         torch.from_numpy(out["sample_ids"]), L, T, train=False)
    err = (lg - torch.from_numpy(out["logits"])).abs().max().item()
    print(f"{name}: N={len(iy)} d={d} V={V} loss={out['loss']:.4f} oracle|d|={err:.2e}")
    assert err < 1e-3


if __name__ == "__main__":
    torch.set_num_threads(8)
    sup_case("mutag_sup", "MUTAG", False, bs=4, k=4, T=1, ff=128, L=1)
    sup_case("mutag_sup_L2T2", "MUTAG", False, bs=4, k=4, T=2, ff=128, L=2)
    sup_case("imdbb_sup", "IMDBBINARY", True, bs=4, k=8, T=4, ff=1024, L=1)
    sampler_case()
    sampled_softmax_case()
    unsup_case()
