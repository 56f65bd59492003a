"""u2gnn_hip — MI355X (gfx950) native U2GNN hot path.

Python host side of the drop-in boundary: ctypes binding of the C ABI (include/*.h),
the forward/backward engine over the HIP kernels, host batch assembly and the
fused optimizer.  The reference-named modules (pytorch_U2GNN_Sup, pytorch_U2GNN_UnSup,
sampled_softmax, log_uniform, util, train_pytorch_U2GNN_*) live one directory up.
"""
from ._lib import U2GNNNativeError, hip_lib, lus_lib  # noqa: F401

__all__ = ["U2GNNNativeError", "hip_lib", "lus_lib"]
