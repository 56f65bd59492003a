"""Micro-benchmark of the fused attention forward (u2gnn_attn_softmax_pv) on C4's shape: the QK^T GEMM
with the EPI_STORE_ROWSTAT epilogue once, then the fused kernel (+ combine) timed over REPS launches with
HIP events, in one process.  Prints avg us per call and the rates the roofline is priced in:
algorithmic FLOPs 2 N^2 d (real dims) and the unique HBM bytes (S read + signed image written).
Usage: python tools/spv_bench.py [N] [d] [p] [prec]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-transformer_amd"))
from u2gnn_hip import _lib  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402
from u2gnn_hip.engine import row_pad  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4776
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 367
    p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
    prec = sys.argv[4] if len(sys.argv) > 4 else "bf16x3"
    reps = int(os.environ.get("SPV_REPS", "20"))
    Np, dp = row_pad(N), (d + 63) // 64 * 64
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    QKV = (torch.randn(Np, 3 * dp, generator=g) * 0.2).to(dev)
    QKV[N:] = 0
    QKV2 = torch.empty(Np, 6 * dp, device=dev, dtype=torch.bfloat16)
    K.split_x2(QKV, 3 * dp, QKV2, 6 * dp, Np, 3 * dp)
    S = torch.empty(Np, Np, device=dev)
    rp = torch.empty(Np, 2 * (Np // 32), device=dev)
    K.gemm(QKV[:, :dp], QKV[:, dp:2 * dp], S, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True,
           epilogue=_lib.EPI_STORE_ROWSTAT, rowpart=rp, n_valid=N, precision=prec, tile=256 if Np % 256 == 0 else 128)
    Pd = torch.empty(Np, Np, device=dev)
    O = torch.empty(Np, dp, device=dev)
    ws = torch.empty(K.attn_softmax_pv_ws_floats(N, Np, dp), device=dev)

    def run():
        K.attn_softmax_pv(S, Np, rp, Np // 64, QKV2, 6 * dp, dp, Pd, Np, O, dp, ws, N, Np, p, 1234, precision=prec)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = 1e3 * e0.elapsed_time(e1) / reps
    fl = 2.0 * N * N * d
    by = 2.0 * 4 * Np * Np
    print(f"spv N={N} d={d} p={p} {prec}: {us:.1f} us/call (fused kernel + combine)  "
          f"{fl / us / 1e6:.1f} TF/s algorithmic  {by / us / 1e3:.0f} GB/s (S + image)")


if __name__ == "__main__":
    main()
