"""Device time of the neighbour-mode window-attention kernels at C4 neighbour shapes (n nodes x W =
k+1 slots, dp = 384), REPS launches captured in one HIP graph.  Run against ablation builds
(tools/build_variant.sh NAME -DU2GNN_EXP_WIN_NODOTS / -DU2GNN_EXP_WIN_NOCOMBINE) through
U2GNN_HIP_LIB.  Usage: python tools/win_bench.py"""
import math
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402

REPS = 20


def t(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(REPS):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


def main():
    n, W, dp = 4864, 17, 384
    rows = n * W
    rows_pad = (rows + 255) // 256 * 256
    g = torch.Generator(device="cuda").manual_seed(0)
    QKV = torch.randn(rows_pad, 3 * dp, device="cuda", generator=g)
    O = torch.empty(rows_pad, dp, device="cuda")
    Ps = torch.empty(n, W, W, device="cuda")
    dO = torch.randn(rows_pad, dp, device="cuda", generator=g)
    dQKV = torch.empty(rows_pad, 3 * dp, device="cuda")
    fwd = t(lambda: K.window_attn_fwd(QKV, W, dp, O, Ps, 0.5, 7, n, rows_pad))
    bwd = t(lambda: K.window_attn_bwd(QKV, W, dp, dO, Ps, 0.5, 7, 1 / math.sqrt(367), dQKV, n, rows_pad))
    fb = (rows_pad * 3 * dp + rows_pad * dp + n * W * W) * 4
    bb = (rows_pad * 3 * dp + 2 * rows_pad * dp + n * W * W + rows_pad * 3 * dp) * 4
    print(f"lib={os.environ.get('U2GNN_HIP_LIB', 'default')}: fwd {fwd:.1f} us ({fb / fwd / 1e3:.0f} GB/s of "
          f"{fb / 1e6:.0f} MB)  bwd {bwd:.1f} us ({bb / bwd / 1e3:.0f} GB/s of {bb / 1e6:.0f} MB)", flush=True)


if __name__ == "__main__":
    main()
