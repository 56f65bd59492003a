"""Generate tests/golden/ptc_unsup_eval.npz: the 10-fold accuracies of the UnSup evaluation
(train_pytorch_U2GNN_UnSup.py:164-188) for a fixed ss.weight on PTC, from the REFERENCE's own pieces:
util.load_data and util.separate_data_idx (util.py:54-158, 176-186) and get_graphpool over ALL graphs
(train_pytorch_U2GNN_UnSup.py:74-94; the same function of the Sup trainer, taken from an executed run of
train_pytorch_U2GNN_Sup.py, since the UnSup script itself cannot be executed: SURVEY.md §0.3).  The body
of evaluate() -- torch.spmm(graph_pool, W), then per fold LogisticRegression(solver="liblinear", tol=0.001)
fit / score -- is restated line for line below (it lives in the unrunnable script).  util.py's module-level
`import pyriemann` (util.py:5; used only by get_gm, out of scope) is satisfied by an empty in-memory module.
The weight is regenerated from its seed (numpy RandomState), so the fixture holds only seed, shape and the
expected accuracies.  The oracle restatement (oracle.u2gnn_oracle.unsup_evaluate) must give the same
numbers (tests/test_unsup_eval.py).  Usage:  python tests/golden/make_eval_golden.py"""
import os
import runpy
import sys
import tempfile
import types

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/U2GNN_pytorch"
sys.modules.setdefault("pyriemann", types.ModuleType("pyriemann"))
sys.path.insert(0, REF)


def weight(seed, V, D):
    return np.random.RandomState(seed).standard_normal((V, D)).astype(np.float32)


def main():
    from sklearn.linear_model import LogisticRegression
    tmp = tempfile.mkdtemp(prefix="u2gnn_ref_")
    sys.argv = ["train_pytorch_U2GNN_Sup.py", "--dataset", "PTC", "--num_epochs", "0", "--ff_hidden_size", "32",
                "--run_folder", os.path.join(tmp, "x") + "/"]
    g = runpy.run_path(os.path.join(REF, "train_pytorch_U2GNN_Sup.py"), run_name="__reference__")
    graphs, separate_data_idx, get_graphpool = g["graphs"], g["separate_data_idx"], g["get_graphpool"]
    graph_labels = np.array([graph.label for graph in graphs])
    graph_pool = get_graphpool(graphs)
    V, D, seed = int(graph_pool.size()[1]), 19, 2024
    node_embeddings = torch.from_numpy(weight(seed, V, D))
    graph_embeddings = torch.spmm(graph_pool, node_embeddings).data.cpu().numpy()
    accs = []
    for fold_idx in range(10):   # evaluate(), train_pytorch_U2GNN_UnSup.py:170-180
        train_idx, test_idx = separate_data_idx(graphs, fold_idx)
        cls = LogisticRegression(solver="liblinear", tol=0.001)
        cls.fit(graph_embeddings[train_idx], graph_labels[train_idx])
        accs.append(cls.score(graph_embeddings[test_idx], graph_labels[test_idx]))
    np.savez(os.path.join(HERE, "ptc_unsup_eval.npz"), seed=seed, V=V, D=D, acc=np.asarray(accs))
    print("accuracies", accs, "mean", np.mean(accs))


if __name__ == "__main__":
    main()
