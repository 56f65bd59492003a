"""Split-K slab reduction micro-benchmark on the layer's shapes: device time of u2gnn_slab_reduce
(HIP events around a HIP-graph replay of back-to-back calls, slabs rewritten before each call as the GEMM leaves them; the
rewrite's own time is subtracted) and its effective
bandwidth.  Usage: python tools/slab_bench.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402

SHAPES = [  # name, slabs, rows_pad, cols_pad, (rblk_pad, rblk_real), accumulate
    ("P.V/dV/dK", 4, 4864, 384, (4864, 4864), 0),
    ("dQ acc", 4, 4864, 384, (4864, 4864), 1),
    ("dWin", 16, 1152, 384, (384, 367), 0),
    ("dW1", 16, 1024, 384, (1024, 1024), 0),
    ("P.V C2", 4, 256, 128, (256, 256), 0),
]
REPS = 50

for name, ns, R, Cc, rb, acc in SHAPES:
    src = torch.randn(ns, R, Cc, device="cuda")
    dst = torch.zeros(rb[1] * (R // rb[0]), Cc, device="cuda")
    f = lambda: K.slab_reduce(src, ns, R * Cc, R, Cc, Cc, rb, (Cc, Cc), dst, Cc, 0.5, acc)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    def timed(with_reduce):   # REPS (slab rewrite [+ reduce]) pairs replayed from one HIP graph
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(REPS):
                src.mul_(1.0)      # rewrite the slabs, as the producing GEMM does
                if with_reduce:
                    f()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / REPS * 1e3
    us = timed(True) - timed(False)
    ref = 0.5 * src.sum(0)
    if rb[0] != rb[1]:
        ref = ref.view(R // rb[0], rb[0], Cc)[:, :rb[1]].reshape(-1, Cc)
    got = dst.clone()
    if acc:
        dst.zero_(); f(); torch.cuda.synchronize(); got = dst
    err = (got - ref).abs().max().item()
    mb = (ns * R * Cc + dst.numel() * (1 + acc)) * 4 / 1e6
    print(f"{name:10s} slabs={ns:2d} {R}x{Cc}: {us:7.2f} us  {mb / us:6.2f} TB/s  maxerr {err:.1e}")
