"""Parity of the HIP sampled-softmax loss and the unsupervised U2GNN (C3 PTC composite) against
golden fixtures generated from the REFERENCE encoder + REFERENCE SampledSoftmax + REFERENCE sampler.
Tolerance: max|ours-ref| / max(1, |ref|) <= 1e-3."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(a, b, tol=1e-3):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item() <= tol


def test_sampled_softmax_vs_reference(golden_dir):
    from sampled_softmax import SampledSoftmax
    z = dict(np.load(os.path.join(golden_dir, "sampled_softmax.npz")))
    V, D = z["weight"].shape
    ss = SampledSoftmax(V, 512, D, DEV).to(DEV)
    ss.weight.data.copy_(torch.from_numpy(z["weight"]))
    x = torch.from_numpy(z["inputs"]).to(DEV).requires_grad_(True)
    labels = torch.from_numpy(z["labels"]).to(DEV)
    logits = ss.sampled(x, labels, (z["sample_ids"], None, None))
    assert close(logits.detach(), z["logits"])
    logits.sum().backward()
    assert close(x.grad, z["grad_inputs"])
    assert close(ss.weight.grad, z["grad_weight"])


def _unsup_model(z):
    from pytorch_U2GNN_UnSup import TransformerU2GNN
    bs, k, T, ff, L, d, V = [int(x) for x in z["meta"]]
    m = TransformerU2GNN(vocab_size=V, feature_dim_size=d, ff_hidden_size=ff, sampled_num=512, num_self_att_layers=T,
                         num_U2GNN_layers=L, dropout=0.5, device=DEV)
    sd = m.state_dict()
    for kk in list(sd):
        if "init." + kk in z:
            sd[kk] = torch.from_numpy(z["init." + kk])
    m.load_state_dict(sd)
    return m.to(DEV).eval(), (bs, k, T, ff, L, d, V)


def test_unsup_module_forward_backward(golden_dir):
    from u2gnn_hip.core import DeviceBatch
    z = dict(np.load(os.path.join(golden_dir, "ptc_unsup.npz")))
    m, _ = _unsup_model(z)
    b = DeviceBatch.from_offsets(z["input_x"], z["offsets"], z["X"], input_y=z["input_y"], device=DEV)
    m.ss.draw_samples = lambda: z["sample_ids"]
    logits, _ = m(b, None, None)
    assert close(logits.detach(), z["logits"])
    logits.sum().backward()
    for n, p in m.named_parameters():
        if "grad." + n in z:
            assert close(p.grad, z["grad." + n]), n


def test_unsup_fused_trainer_step(golden_dir):
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.unsup import UnSupTrainer
    z = dict(np.load(os.path.join(golden_dir, "ptc_unsup.npz")))
    m, _ = _unsup_model(z)
    tr = UnSupTrainer(m, lr=float(z["lr"]))
    b = DeviceBatch.from_offsets(z["input_x"], z["offsets"], z["X"], input_y=z["input_y"], device=DEV)
    sid = torch.from_numpy(z["sample_ids"]).to(DEV)
    loss = tr.step(b, sid, train=False)
    assert abs(loss.item() - float(z["loss"])) <= 1e-3 * max(1.0, abs(float(z["loss"])))
    assert abs(tr.opt.grad_norm() - float(z["grad_norm"])) <= 1e-3 * float(z["grad_norm"])
    for n, p in m.named_parameters():
        if "after." + n in z:
            assert close(p.detach(), z["after." + n]), n


def test_unsup_forward_backward_twice_leaves_one_batch_gradient(golden_dir):
    """a second forward_backward without step()/clear_row_grads() in between (an evaluation
    loss, a gradient check) must leave exactly ONE batch's ss.weight gradient -- the rows the first
    call added are zeroed, not carried into every later clip norm and Adam update."""
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.unsup import UnSupTrainer
    z = dict(np.load(os.path.join(golden_dir, "ptc_unsup.npz")))
    m, _ = _unsup_model(z)
    tr = UnSupTrainer(m, lr=float(z["lr"]))
    b = DeviceBatch.from_offsets(z["input_x"], z["offsets"], z["X"], input_y=z["input_y"], device=DEV)
    sid = torch.from_numpy(z["sample_ids"]).to(DEV)
    other = torch.from_numpy((z["sample_ids"] + 17) % int(z["meta"][-1])).to(DEV)
    tr.forward_backward(b, other, train=False)          # rows this call touches differ from the next
    tr.forward_backward(b, sid, train=False)
    twice = tr.flat.gflat.clone()
    tr.clear_row_grads()
    assert tr.flat.grads["ss.weight"].abs().max().item() == 0.0
    tr.forward_backward(b, sid, train=False)
    assert torch.equal(twice, tr.flat.gflat)
    assert close(tr.flat.grads["ss.weight"], z["grad.ss.weight"])


def test_graph_embeddings_match_spmm_over_all_graphs():
    """evaluate() of train_pytorch_U2GNN_UnSup.py:167-169: spmm(graph_pool, ss.weight) with graph_pool
    built over ALL graphs (train_pytorch_U2GNN_UnSup.py:92-94) -- the per-graph sums of the learned
    node embeddings, here against a float64 torch.sparse reference on the PTC node layout."""
    import util
    from u2gnn_hip.batching import GraphStore
    from u2gnn_hip.unsup import graph_embeddings
    graphs, _ = util.load_data("PTC", False)
    store = GraphStore(graphs)
    V = int(store.node_start[-1])
    g = torch.Generator(device="cuda").manual_seed(11)
    for D in (19, 4, 64):
        W = torch.randn(V, D, device="cuda", generator=g)
        emb = graph_embeddings(W, store.node_start)
        rows = np.repeat(np.arange(len(graphs)), np.diff(store.node_start))
        pool = torch.sparse_coo_tensor(torch.tensor(np.stack([rows, np.arange(V)])), torch.ones(V, dtype=torch.float64),
                                       (len(graphs), V))
        ref = torch.sparse.mm(pool, W.double().cpu())
        assert emb.shape == (len(graphs), D)
        assert ((emb.double().cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-6
