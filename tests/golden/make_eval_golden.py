"""Generate tests/golden/ptc_unsup_eval.npz: the 10-fold accuracies of the UnSup evaluation
(train_pytorch_U2GNN_UnSup.py:164-188) for a fixed ss.weight on PTC, computed by the oracle's
restatement (oracle.u2gnn_oracle.unsup_evaluate: torch.spmm over graph_pool of ALL graphs +
LogisticRegression(liblinear, tol=1e-3) on the StratifiedKFold(10, shuffle, seed 0) splits).  The
weight is regenerated from its seed (numpy RandomState), so the fixture holds only seed, shape and
the expected accuracies.  Usage:  python tests/golden/make_eval_golden.py"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)

from oracle import u2gnn_oracle as O  # noqa: E402


def weight(seed, V, D):
    return np.random.RandomState(seed).standard_normal((V, D)).astype(np.float32)


def main():
    graphs, _ = O.load_data(os.path.join(REPO, "dataset", "PTC", "PTC.txt"), False)
    n = [g.n for g in graphs]
    labels = [g.label for g in graphs]
    V, D, seed = int(sum(n)), 19, 2024
    accs = O.unsup_evaluate(torch.from_numpy(weight(seed, V, D)), n, labels)
    np.savez(os.path.join(HERE, "ptc_unsup_eval.npz"), seed=seed, V=V, D=D, acc=np.asarray(accs))
    print("accuracies", accs, "mean", np.mean(accs))


if __name__ == "__main__":
    main()
