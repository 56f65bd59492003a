"""UnSup evaluation (train_pytorch_U2GNN_UnSup.py:164-188): graph embeddings =
spmm(graph_pool over ALL graphs, ss.weight), then 10-fold LogisticRegression(liblinear, tol=1e-3).
Pinned by tests/golden/ptc_unsup_eval.npz (tests/golden/make_eval_golden.py: the oracle's
restatement on PTC for a seeded ss.weight).  CPU: the oracle and the product's host half
(util.separate_data_idx + unsup.fold_accuracies) reproduce the fixture exactly.  GPU: the product's
device embeddings (u2gnn_pool_fwd over all graphs) give the same accuracies; fp32 sums in another
order may move a test graph across the decision boundary, so at most one test graph per fold may
differ."""
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _case():
    z = dict(np.load(os.path.join(HERE, "golden", "ptc_unsup_eval.npz")))
    seed, V, D = int(z["seed"]), int(z["V"]), int(z["D"])
    W = np.random.RandomState(seed).standard_normal((V, D)).astype(np.float32)
    return W, z["acc"]


def _ptc():
    import util
    graphs, _ = util.load_data("PTC", False)
    labels = np.array([g.label for g in graphs])
    folds = [util.separate_data_idx(graphs, i) for i in range(10)]
    return graphs, labels, folds


def test_oracle_evaluation_reproduces_fixture():
    from oracle import u2gnn_oracle as O
    W, acc = _case()
    graphs, labels, _ = _ptc()
    got = O.unsup_evaluate(torch.from_numpy(W), [len(g.g) if hasattr(g, "g") else g.n for g in graphs], labels)
    assert np.array_equal(np.asarray(got), acc)


def test_product_fold_accuracies_on_host_embeddings():
    from u2gnn_hip.batching import GraphStore
    from u2gnn_hip.unsup import fold_accuracies
    W, acc = _case()
    graphs, labels, folds = _ptc()
    start = GraphStore(graphs).node_start
    rows = np.repeat(np.arange(len(graphs)), np.diff(start))
    pool = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, np.arange(int(start[-1]))])),
                                   torch.ones(int(start[-1])), (len(graphs), int(start[-1])))
    emb = torch.spmm(pool, torch.from_numpy(W)).numpy()
    assert np.array_equal(np.asarray(fold_accuracies(emb, labels, folds)), acc)


@pytest.mark.gpu
def test_device_embeddings_evaluation_matches_fixture():
    from u2gnn_hip.batching import GraphStore
    from u2gnn_hip.unsup import fold_accuracies, graph_embeddings
    W, acc = _case()
    graphs, labels, folds = _ptc()
    start = GraphStore(graphs).node_start
    emb = graph_embeddings(torch.from_numpy(W).cuda(), start).cpu().numpy()
    got = np.asarray(fold_accuracies(emb, labels, folds))
    one = np.array([1.0 / len(te) for _, te in folds])
    assert np.all(np.abs(got - acc) <= one + 1e-12), (got, acc)
    assert np.sum(got != acc) <= 2
