"""Micro-benchmark of a whole small-width encoder layer (u2gnn_layer_small_fwd / _bwd, csrc/small_layer.hip) on C5-like
shapes (d = 4, ff = 1024, N ~ 2 K rows): device time per call via HIP events over back-to-back launches replayed from
a captured graph.  Usage: python tools/small_layer_bench.py [reps]   (U2GNN_HIP_LIB selects a variant library)"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402
from u2gnn_hip.engine import row_pad  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
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
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = "cuda"
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    tag = os.path.basename(os.environ.get("U2GNN_HIP_LIB", "default"))
    shapes = ((1914, 4, 1024), (3900, 4, 1024), (700, 7, 1024))
    for N, d, ff in shapes[:int(os.environ.get("SLB_SHAPES", len(shapes)))]:
        Np, dp, ffp = row_pad(N), 64, -(-ff // 64) * 64
        g = torch.Generator(device=dev).manual_seed(N)
        rn = lambda *s: torch.randn(*s, device=dev, generator=g)   # noqa: E731
        W_in, b_in = torch.zeros(3 * dp, dp, device=dev), torch.zeros(3 * dp, device=dev)
        for k in range(3):
            W_in[k * dp:k * dp + d, :d] = rn(d, d) * 0.5
        w = dict(W_o=torch.zeros(dp, dp, device=dev), b_o=torch.zeros(dp, device=dev), n1_w=torch.ones(d, device=dev),
                 n1_b=torch.zeros(d, device=dev), W1=torch.zeros(ffp, dp, device=dev), b1=0.1 * rn(ffp),
                 W2=torch.zeros(dp, ffp, device=dev), b2=torch.zeros(dp, device=dev), n2_w=torch.ones(d, device=dev),
                 n2_b=torch.zeros(d, device=dev))
        w["W_o"][:d, :d] = rn(d, d)
        w["W1"][:ff, :d] = rn(ff, d)
        w["W2"][:d, :ff] = rn(d, ff) * 0.05
        X = torch.zeros(Np, dp, device=dev)
        X[:N, :d] = rn(N, d)
        fw = {k: torch.zeros(Np, c, device=dev) for k, c in (("O", dp), ("Z1", dp), ("X1", dp), ("Hd", ffp), ("Z2", dp),
                                                              ("X2", dp))}
        fw.update({k: torch.zeros(Np, device=dev) for k in ("mean1", "rstd1", "mean2", "rstd2")})
        ctx = torch.zeros(K.attn_small_ctx_floats(Np, d), device=dev)
        bw = {k: torch.zeros(Np, c, device=dev) for k, c in (("dX1", dp), ("dF", dp), ("dH", ffp), ("dX", dp),
                                                              ("dA", dp), ("dO", dp))}
        bw["delta"] = torch.zeros(Np, device=dev)
        dX2 = torch.zeros(Np, dp, device=dev)
        dX2[:N, :d] = rn(N, d)
        dQKV = torch.zeros(Np, 3 * dp, device=dev)
        ws = torch.zeros(K.attn_small_ws_floats(N, Np, d), device=dev)
        fw_in = {k: v for k, v in fw.items() if k != "X2"}

        def fwd():
            K.layer_small_fwd(N, Np, d, dp, ff, ffp, 0.5, (1, 2, 3), 4, W_in, b_in, ctx, X=X, **w, **fw)

        def bwd():
            K.layer_small_bwd(N, Np, d, dp, ff, ffp, 0.5, (1, 2, 3), 4, W_in, ctx, dQKV, True, ws, dX2=dX2, X=X,
                              **w, **fw_in, **bw)
        print(f"{tag} N={N:5d} d={d:2d} ff={ff}  fwd {timed(fwd, reps):7.1f} us  bwd {timed(bwd, reps):7.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
