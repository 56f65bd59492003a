"""Reference ceiling (not product code): hipBLASLt via torch.matmul on the bf16 shapes a library
bf16x3 formulation of the C4 attention products would run ([N, 3d] x [3d, N] and [N, 3N] x [3N, d]),
next to this repo's own kernels in plain bf16 and bf16x3 on the same products.
Usage: python tools/blas_ceiling.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402

Np, dp, N, d = 4864, 384, 4776, 367


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    bf = torch.bfloat16
    A = torch.randn(Np, 3 * dp, device="cuda", generator=g).to(bf)
    B = torch.randn(3 * dp, Np, device="cuda", generator=g).to(bf)
    t = timeit(lambda: A @ B)
    fl_alg = 2.0 * N * N * d
    print(f"hipBLASLt bf16 [Np,3dp]x[3dp,Np] {t:7.1f} us  {2.0 * Np * Np * 3 * dp / t / 1e6:7.1f} TF raw  "
          f"{fl_alg / t / 1e6:6.1f} TF algorithmic (x3)", flush=True)
    Bt = B.t().contiguous()
    t = timeit(lambda: A @ Bt.t())
    print(f"hipBLASLt bf16 NT                {t:7.1f} us  {2.0 * Np * Np * 3 * dp / t / 1e6:7.1f} TF raw", flush=True)
    A2 = torch.randn(Np, 3 * Np, device="cuda", generator=g).to(bf)
    B2 = torch.randn(3 * Np, dp, device="cuda", generator=g).to(bf)
    t = timeit(lambda: A2 @ B2)
    print(f"hipBLASLt bf16 [Np,3Np]x[3Np,dp] {t:7.1f} us  {2.0 * Np * dp * 3 * Np / t / 1e6:7.1f} TF raw  "
          f"{fl_alg / t / 1e6:6.1f} TF algorithmic (x3)", flush=True)
    Q = torch.randn(Np, dp, device="cuda", generator=g)
    Kt = torch.randn(Np, dp, device="cuda", generator=g)
    S = torch.empty(Np, Np, device="cuda")
    for prec in ("bf16", "bf16x3"):
        t = timeit(lambda: K.gemm(Q, Kt, S, Np, Np, dp, dp, dp, Np, trans_b=True, precision=prec, tile=256))
        mult = 3 if prec == "bf16x3" else 1
        print(f"u2gnn {prec:6s} QK^T                {t:7.1f} us  {2.0 * Np * Np * dp * mult / t / 1e6:7.1f} "
              f"TF MFMA-equivalent", flush=True)
    Q16, K16 = Q.to(bf), Kt.to(bf)
    t = timeit(lambda: Q16 @ K16.t())
    print(f"hipBLASLt bf16 QK^T (K=dp)       {t:7.1f} us  {2.0 * Np * Np * dp / t / 1e6:7.1f} TF raw", flush=True)
    Af = torch.randn(Np, 3 * dp, device="cuda", generator=g)
    Bf = torch.randn(3 * dp, Np, device="cuda", generator=g)
    t = timeit(lambda: Af @ Bf)
    print(f"hipBLASLt fp32 [Np,3dp]x[3dp,Np] {t:7.1f} us  {2.0 * Np * Np * 3 * dp / t / 1e6:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
