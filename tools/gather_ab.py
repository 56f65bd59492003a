"""A/B of the a2 gather variants (U2GNN_GATHER_MODE=0|2, read once per process) on one C4 batch:
bit-exact check against torch indexing, then bench.py's gather_roofline timing.
Usage: for m in 0 2; do U2GNN_GATHER_MODE=$m python tools/gather_ab.py; done"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402
from u2gnn_hip.batching import BatchLoader  # noqa: E402
from u2gnn_hip.core import DeviceBatch  # noqa: E402
from u2gnn_hip.engine import Dims, rup  # noqa: E402
from u2gnn_hip.synthetic import collab_like  # noqa: E402

BS = int(os.environ.get("GA_BATCH", "64"))


def main():
    dev = torch.device("cuda", 0)
    np.random.seed(0)
    hb = BatchLoader(collab_like(seed=0), BS, 16)()
    b = DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels, device=dev)
    d = b.X_concat.shape[1]
    W = b.input_x.shape[1]
    R = b.N * W
    Rp, dp = Dims(R, d, 1024).Np, rup(d, 64)
    dst = torch.full((Rp, dp), float("nan"), device=dev)
    K.gather_rows(b.X_concat, b.input_x, 1, dst, R, Rp, d, dp)
    ref = torch.zeros(Rp, dp, device=dev)
    ref[:R, :d] = b.X_concat[b.input_x.reshape(-1)]
    exact = torch.equal(dst, ref)
    r = bench.gather_roofline(b, d, 1024, K, dev, reps=50)
    print(f"mode={os.environ.get('U2GNN_GATHER_MODE', '0')} exact={exact} us={r['avg_launch_us']} "
          f"GB/s={r['achieved']} frac={r['frac']} R={R} Rp={Rp} dp={dp}", flush=True)
    assert exact
    if os.environ.get("GA_CEIL"):
        def t(fn, reps=50):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps
        other = torch.randn_like(dst)
        tz, tc = t(dst.zero_), t(lambda: dst.copy_(other))
        nb = dst.numel() * 4
        print(f"ceiling: fill {tz:.2f} us {nb / tz / 1e3:.0f} GB/s (write) | copy {tc:.2f} us "
              f"{2 * nb / tc / 1e3:.0f} GB/s (r+w)", flush=True)


if __name__ == "__main__":
    main()
