"""SURVEY §8(d) CPU-baseline cross-check, run in the build container (not on the GPU box, where the
reference does not exist): the oracle restatement that bench.py times as `cpu_baseline` against the
REFERENCE model itself (pytorch_U2GNN_Sup.TransformerU2GNN imported from /root/reference by file path,
torch-only import; the reference's train-step body of train_pytorch_U2GNN_Sup.py:146-160), on the same
C4 batch, same initial weights, all host cores.  Reports the median of --steps steps of each and the
ratio (the survey's bar: within +-15 %).
Usage: python tools/cpu_crosscheck.py [--steps 3] [--out profiles/r03/cpu_crosscheck.json]"""
import argparse
import importlib.util
import json
import os
import platform
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "graph-transformer_amd")]
REF_FILE = "/root/reference/U2GNN_pytorch/pytorch_U2GNN_Sup.py"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.machine()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "cpu_crosscheck.json"))
    args = ap.parse_args()
    from oracle import u2gnn_oracle as O
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.synthetic import collab_like

    threads = os.cpu_count() or 1
    torch.set_num_threads(threads)
    d, C, ff, T, L = 367, 3, 1024, 4, 1
    store = collab_like(seed=0)
    np.random.seed(123)
    hb = BatchLoader(store, 64, 16)()
    spec = importlib.util.spec_from_file_location("reference_pytorch_U2GNN_Sup", REF_FILE)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    torch.manual_seed(123)
    model = ref.TransformerU2GNN(feature_dim_size=d, ff_hidden_size=ff, num_classes=C, num_self_att_layers=T,
                                 dropout=0.5, num_U2GNN_layers=L).train()
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ix = torch.from_numpy(hb.input_x)
    X = torch.from_numpy(hb.X_concat)
    lab = torch.from_numpy(hb.labels)
    B = lab.shape[0]
    off = np.asarray(hb.offsets)
    rows = np.repeat(np.arange(B), np.diff(off))
    idx = torch.from_numpy(np.stack([rows, np.arange(off[-1])]).astype(np.int64))
    pool = torch.sparse_coo_tensor(idx, torch.ones(idx.shape[1]), (B, int(off[-1])))
    target = ref.label_smoothing(lab, C)

    def ref_step(opt):
        opt.zero_grad()
        scores = model(ix, pool, X)
        loss = torch.mean(torch.sum(-target * torch.log_softmax(scores, dim=1), 1))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()

    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    plist = list(params.values())
    opt_o = torch.optim.Adam(plist, lr=5e-4)

    def oracle_step():
        opt_o.zero_grad()
        scores = O.sup_forward(params, ix, hb.offsets, X, L, T, train=True, dropout=0.5)
        loss = O.soft_cross_entropy(scores, O.label_smoothing(lab, C))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(plist, 0.5)
        opt_o.step()

    opt_r = torch.optim.Adam(model.parameters(), lr=5e-4)
    t_ref, t_orc = [], []
    for _ in range(args.steps):   # interleaved: the two see the same machine state
        t0 = time.perf_counter()
        ref_step(opt_r)
        t_ref.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        oracle_step()
        t_orc.append(time.perf_counter() - t0)
        print(f"reference {t_ref[-1]:.1f} s, oracle {t_orc[-1]:.1f} s", flush=True)
    mr, mo = float(np.median(t_ref)), float(np.median(t_orc))
    out = {"what": "one C4 training step (64 graphs, all 17 slots, dropout on, clip + Adam) on torch CPU",
           "batch_nodes": int(off[-1]), "threads": threads, "cpu": cpu_model(),
           "reference_step_s": [round(x, 2) for x in t_ref], "oracle_step_s": [round(x, 2) for x in t_orc],
           "reference_graphs_per_s": round(B / mr, 3), "oracle_graphs_per_s": round(B / mo, 3),
           "oracle_over_reference_time": round(mo / mr, 3), "bar": "within +-15 % (SURVEY §8(d))",
           "within_bar": bool(abs(mo / mr - 1.0) <= 0.15)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
