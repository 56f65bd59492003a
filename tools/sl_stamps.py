"""Phase timing of the fused small-width layer kernels (sa_fwd_kernel / sa_bwd_q_kernel with TAIL) from in-kernel
wall-clock stamps: build the variant with  bash tools/build_variant.sh stamps -DSX_STAMPS  and run
U2GNN_HIP_LIB=$PWD/graph-transformer_amd/lib/exp_stamps.so python tools/sl_stamps.py
Prints, per phase boundary, the median / max over workgroups of the time since the kernel's first stamp (us)."""
import ctypes
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd"),
                os.path.dirname(os.path.abspath(__file__))]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import small_layer_bench as B  # noqa: E402
from u2gnn_hip import _lib  # noqa: E402

NAMES = {0: ["start", "tile0 staged", "walk done", "merge+sync", "O written", "LN1+sync", "W chunk staged",
             "FFN done", "z2 sums+sync", "end"],
         1: ["start", "tail done", "tile0 staged", "walk done", "end", "LN2T+sync", "W chunk staged", "FFN done",
             "dx1 sums+sync"]}


def main():
    os.environ["SLB_SHAPES"] = "1"
    B.main()   # warm-up and timing (prints)
    lib = _lib.hip_lib()
    buf = np.zeros((2, 4096, 16), dtype=np.uint64)
    torch.cuda.synchronize()
    rc = lib.u2gnn_dbg_sx_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.size))
    assert rc == 0, rc
    for kern in (0, 1):
        st = buf[kern].astype(np.float64)
        used = st[:, 0] > 0
        st = st[used]
        t0 = st[:, 0].min()
        print(f"kernel {'fwd' if kern == 0 else 'bwd_q'}: {used.sum()} workgroups, stamps in us since the first start")
        for k, name in enumerate(NAMES[kern]):
            col = (st[:, k] - t0) / 100.0
            ok = st[:, k] > 0
            if ok.any():
                col = col[ok]
                print(f"  {k} {name:16s} min {col.min():7.2f} med {np.median(col):7.2f} max {col.max():7.2f}")


if __name__ == "__main__":
    main()
