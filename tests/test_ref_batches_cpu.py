"""Rows a1 (batch assembly, neighbour sampling) and f2 (GIN loader, tag map, fold split) against fixtures
produced by RUNNING THE REFERENCE (tests/golden/make_ref_batches.py: train_pytorch_U2GNN_Sup.py executed
with its own util.load_data / separate_data / Batch_Loader / get_batch_data on the seed-123 stream).

Bit-exact: every graph's node count, label, tag index and edge list in file order (util.py:54-158); the
fold-1 split (util.py:160-173); input_x, offsets, labels and the one-hot tag of every row of the first
training batches (train_pytorch_U2GNN_Sup.py:91-128) and of the evaluation batches that follow on the same
stream (:166-179); the unsupervised batches' input_x, selections and input_y
(train_pytorch_U2GNN_UnSup.py:96-134).  The product path is the CLI's: util.load_data, separate_data,
GraphStore + BatchLoader (native C++ assembly, csrc/batch_assembly.cpp), and the numpy form beside it."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _z(name):
    return dict(np.load(os.path.join(GOLDEN, f"ref_batches_{name}.npz")))


def _check_loader(z, graphs):
    assert len(graphs) == len(z["g_n_nodes"])
    assert graphs[0].node_features.shape[1] == int(z["g_d"])
    n = np.array([g.n if hasattr(g, "n") else len(g.g) for g in graphs])
    assert np.array_equal(n, z["g_n_nodes"])
    assert np.array_equal(np.array([g.label for g in graphs]), z["g_labels"])
    assert np.array_equal(np.concatenate([np.argmax(g.node_features, 1) for g in graphs]), z["g_tag"])
    edges = np.concatenate([np.asarray(g.edge_mat, np.int64).reshape(2, -1) for g in graphs], 1)
    assert np.array_equal(np.array([np.asarray(g.edge_mat).reshape(2, -1).shape[1] for g in graphs]), z["g_n_edges"])
    assert np.array_equal(edges, z["g_edges"])


def _check_batch(z, p, hb):
    assert np.array_equal(hb.input_x, z[p + "input_x"]), p
    assert np.array_equal(np.asarray(hb.offsets), z[p + "offsets"]), p
    assert np.array_equal(np.argmax(hb.X_concat, 1), z[p + "tag"]), p
    if p + "labels" in z and p.startswith("b"):
        assert np.array_equal(np.asarray(hb.labels), z[p + "labels"]), p


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("name,dataset,deg_tag", [("mutag", "MUTAG", False), ("imdbb", "IMDBBINARY", True)])
def test_sup_loader_split_and_batches_equal_the_reference_run(name, dataset, deg_tag, native):
    import util
    from u2gnn_hip.batching import BatchLoader, GraphStore
    z = _z(name)
    bs, k, nb = [int(x) for x in z["meta"]]
    np.random.seed(123)                     # train_pytorch_U2GNN_Sup.py:9, as the CLI does
    graphs, _ = util.load_data(dataset, deg_tag)
    _check_loader(z, graphs)
    tr, te = util.separate_data_idx(graphs, 1)
    assert np.array_equal(np.asarray(tr), z["train_idx"]) and np.array_equal(np.asarray(te), z["test_idx"])
    train, test = util.separate_data(graphs, 1)
    loader = BatchLoader(GraphStore(train), bs, k, native=native)
    for i in range(nb):
        _check_batch(z, f"b{i}_", loader())
    test_store = GraphStore(test)
    idx = np.arange(len(test))
    for e, i in enumerate(range(0, len(test), bs)):   # evaluate(): test graphs in order, same stream
        sel = idx[i:i + bs]
        hb = test_store.assemble(sel, k) if native else test_store.assemble_numpy(sel, k)
        _check_batch(z, f"e{e}_", hb)
    assert e + 1 == int(z["n_eval"])


@pytest.mark.parametrize("native", [True, False])
def test_unsup_batches_equal_the_reference_run(native):
    import util
    from u2gnn_hip.batching import BatchLoader, GraphStore
    z = _z("ptc_unsup")
    bs, k, nb = [int(x) for x in z["meta"]]
    np.random.seed(123)
    graphs, _ = util.load_data("PTC", False)
    _check_loader(z, graphs)
    loader = BatchLoader(GraphStore(graphs), bs, k, with_input_y=True, native=native)
    for i in range(nb):
        hb = loader()
        _check_batch(z, f"b{i}_", hb)
        assert np.array_equal(np.asarray(hb.graph_ids), z[f"b{i}_sel"])
        assert np.array_equal(hb.input_y, z[f"b{i}_input_y"])
