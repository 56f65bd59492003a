"""u2gnn_hip — MI355X (gfx950) native U2GNN hot path.

Python host side of the drop-in boundary: ctypes binding of the C ABI (include/*.h),
the forward/backward engine over the HIP kernels, host batch assembly and the
fused optimizer.  The reference-named modules (pytorch_U2GNN_Sup, pytorch_U2GNN_UnSup,
sampled_softmax, log_uniform, util, train_pytorch_U2GNN_*) live one directory up.
"""
import os as _os


def ensure_hw_queues(n: int = 8) -> None:
    """Give this process at least `n` HIP hardware queues (GPU_MAX_HW_QUEUES; HIP's default is 4).
    The layer executor runs a main and a side stream; once RCCL's communicator adds its own
    streams, 4 queues make the side stream share the main stream's queue and the two serialise
    (measured at C4 with a 1-rank RCCL group: 3.82 ms/step with 4 queues, 3.36 with 8, 3.34
    without RCCL).  Only effective before the HIP runtime initialises, so it runs at import."""
    cur = _os.environ.get("GPU_MAX_HW_QUEUES", "")
    if not cur.isdigit() or int(cur) < n:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(n)


ensure_hw_queues()

from ._lib import U2GNNNativeError, hip_lib, lus_lib  # noqa: F401,E402

__all__ = ["U2GNNNativeError", "hip_lib", "lus_lib"]
