"""GEMM micro-benchmark on the C4 attention / weight-gradient shapes (device time via HIP events).
Usage: python tools/gemm_bench.py [precision ...]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402

Np, dp, ffp = 4864, 384, 1024
SHAPES = [  # name, M, N, K, ta, tb, split, tile
    ("QK^T  NT", Np, Np, dp, False, True, 1, 128),
    ("P.V   NN", Np, dp, Np, False, False, 4, 128),
    ("dV    TN", Np, dp, Np, True, False, 4, 128),
    ("dWin  TN", 3 * dp, dp, Np, True, False, 16, 128),
    ("dW1   TN", ffp, dp, Np, True, False, 16, 128),
    ("QKV   NT", Np, 3 * dp, dp, False, True, 1, 64),
    ("FFN1  NT", Np, ffp, dp, False, True, 1, 64),
    ("FFN2  NT", Np, dp, ffp, False, True, 1, 64),
]


def run(prec):
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, Kd, ta, tb, split, tile in SHAPES:
        A = torch.randn(Kd, M, device="cuda", generator=g) if ta else torch.randn(M, Kd, device="cuda", generator=g)
        B = torch.randn(N, Kd, device="cuda", generator=g) if tb else torch.randn(Kd, N, device="cuda", generator=g)
        C = torch.empty(split, M, N, device="cuda")
        f = lambda: K.gemm(A, B, C, M, N, Kd, A.shape[1], B.shape[1], N, trans_a=ta, trans_b=tb, split_k=split,  # noqa
                           slab_stride=M * N, tile=tile, precision=prec)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        print(f"{prec:7s} {name}  M={M:5d} N={N:5d} K={Kd:5d} split={split:2d} tile={tile:3d}: {us:8.1f} us "
              f"{2.0 * M * N * Kd / us / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    for p in (sys.argv[1:] or ["bf16x3", "fp32"]):
        run(p)
