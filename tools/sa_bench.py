"""Micro-benchmark of the small-width projection + attention kernels (u2gnn_attn_small_fwd / _bwd, csrc/small_layer.hip) on
C5-like shapes (d = 4, N ~ 2 K) and C3 / MUTAG ones: device time per call via HIP events over back-to-back
launches replayed from a captured graph.  Usage: python tools/sa_bench.py   (U2GNN_HIP_LIB selects a variant library)"""
import math
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402
from u2gnn_hip.engine import row_pad  # noqa: E402


def main():
    dev = "cuda"
    reps = 50
    for N, d in ((2034, 4), (4000, 4), (102, 19), (72, 7)):
        Np, dp = row_pad(N), 64
        g = torch.Generator(device=dev).manual_seed(1)
        X = torch.zeros(Np, dp, device=dev)
        X[:N, :d] = torch.randn(N, d, device=dev, generator=g)
        W = torch.zeros(3 * dp, dp, device=dev)
        for b in range(3):
            W[b * dp:b * dp + d, :d] = torch.randn(d, d, device=dev, generator=g) / math.sqrt(d)
        bias = torch.zeros(3 * dp, device=dev)
        dO = torch.zeros(Np, dp, device=dev)
        dO[:N, :d] = torch.randn(N, d, device=dev, generator=g)
        O, ctx = torch.empty(Np, dp, device=dev), torch.empty(K.attn_small_ctx_floats(Np, d), device=dev)
        delta = torch.randn(Np, device=dev, generator=g)
        dQKV, dX = torch.empty(Np, 3 * dp, device=dev), torch.zeros(Np, dp, device=dev)
        ws = torch.empty(max(1, K.attn_small_ws_floats(N, Np, d)), device=dev)

        def fwd():
            K.attn_small_fwd(X, dp, W, bias, dp, d, N, Np, 0.5, 3, O, dp, ctx)

        def bwd():
            K.attn_small_bwd(ctx, W, dp, d, N, Np, 0.5, 3, dO, dp, delta, 1 / math.sqrt(d), dQKV, 3 * dp, dX, dp, ws)
        out = []
        for name, fn in (("fwd", fwd), ("bwd", bwd)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()   # back-to-back launches without the Python call overhead
            with torch.cuda.graph(graph):
                for _ in range(reps):
                    fn()
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
            out.append(f"{name} {e0.elapsed_time(e1) * 1e3 / reps:7.1f} us")
        print(f"N={N:5d} d={d:2d}  " + "  ".join(out), flush=True)


if __name__ == "__main__":
    main()
