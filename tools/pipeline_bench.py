"""End-to-end C4 training throughput INCLUDING host batch assembly: each step
assembles its 64-graph COLLAB-like batch on the host from the real-dataset store (GraphStore over
the synthetic graphs), moves it to the GPU and trains on it.  Three pipelines:
  numpy  : numpy assembly (broadcast randint) + host X_concat + pageable H2D (DeviceBatch.from_offsets)
  native : native assembly (csrc/batch_assembly.cpp) + host X_concat
  native+gpu-gather : native assembly without X; features gathered on the GPU (DeviceBatch.from_store)
bench.py's headline value excludes host assembly (batches resident in HBM); this tool reports what
a training loop that builds its batches on the fly gets.  Usage: python tools/pipeline_bench.py [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), os.path.join(REPO, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import loader_bench  # noqa: E402
from pytorch_U2GNN_Sup import TransformerU2GNN  # noqa: E402
from u2gnn_hip.batching import BatchLoader  # noqa: E402
from u2gnn_hip.core import DeviceBatch  # noqa: E402
from u2gnn_hip.train import SupTrainer  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    store = loader_bench.collab_store()
    X_dev = torch.from_numpy(store.X).to(dev)
    torch.manual_seed(123)
    model = TransformerU2GNN(feature_dim_size=367, ff_hidden_size=1024, num_classes=3, num_self_att_layers=4,
                             dropout=0.5, num_U2GNN_layers=1, precision="bf16x3").to(dev).train()
    trainer = SupTrainer(model, lr=5e-4, max_norm=0.5, seed=123)
    modes = {
        "numpy": (dict(native=False), lambda hb: DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat,
                                                                          hb.labels, device=dev)),
        "native": (dict(), lambda hb: DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels,
                                                               device=dev)),
        "native+gpu-gather": (dict(gather_x=False), lambda hb: DeviceBatch.from_store(hb, X_dev, device=dev)),
    }
    # reference on the same box: pre-assembled batches resident in HBM (what bench.py times)
    np.random.seed(123)
    res_loader = BatchLoader(store, 64, 16)
    resident = [DeviceBatch.from_offsets(h.input_x, h.offsets, h.X_concat, h.labels, device=dev)
                for h in (res_loader() for _ in range(8))]
    for i in range(3):
        trainer.step(resident[i % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        trainer.step(resident[i % 8])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{'resident (bench)':18s} {64 * steps / el:9.1f} graphs/s  {1e3 * el / steps:6.2f} ms/step", flush=True)
    for name, (kw, to_dev) in modes.items():
        np.random.seed(123)
        loader = BatchLoader(store, 64, 16, **kw)
        for _ in range(3):
            trainer.step(to_dev(loader()))
        torch.cuda.synchronize()
        host = xfer = issue = 0.0
        t0 = time.perf_counter()
        for _ in range(steps):
            h0 = time.perf_counter()
            hb = loader()
            h1 = time.perf_counter()
            b = to_dev(hb)
            h2 = time.perf_counter()
            trainer.step(b)
            h3 = time.perf_counter()
            host, xfer, issue = host + h1 - h0, xfer + h2 - h1, issue + h3 - h2
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"{name:18s} {64 * steps / el:9.1f} graphs/s  {1e3 * el / steps:6.2f} ms/step  host per step: "
              f"assembly {1e3 * host / steps:5.2f}, to-device {1e3 * xfer / steps:5.2f}, step issue "
              f"{1e3 * issue / steps:5.2f} ms", flush=True)


if __name__ == "__main__":
    main()
