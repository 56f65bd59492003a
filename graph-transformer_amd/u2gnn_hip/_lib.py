"""ctypes binding of the two native libraries (C ABI: include/u2gnn_hip.h, include/u2gnn_lus.h).

The product path has no CPU fallback: if ``libu2gnn_hip.so`` is missing or cannot be
loaded, every kernel entry point raises ``U2GNNNativeError`` (build it with
``make -C graph-transformer_amd/csrc`` or ``python -c 'import __graft_entry__ as g; g.build()'``).
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_double, c_float, c_int32, c_int64, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_DIR = os.path.join(PKG_ROOT, "lib")
INCLUDE_DIR = os.path.join(REPO_ROOT, "include")
# U2GNN_HIP_LIB: an alternative build of the same kernels (tools/ experiments)
HIP_LIB_PATH = os.environ.get("U2GNN_HIP_LIB") or os.path.join(LIB_DIR, "libu2gnn_hip.so")
LUS_LIB_PATH = os.path.join(LIB_DIR, "libu2gnn_lus.so")


class U2GNNNativeError(RuntimeError):
    pass


# error codes (u2gnn_hip.h)
U2GNN_OK = 0
ERRORS = {-1: "bad argument", -2: "misaligned pointer / leading dimension", -3: "shape not a tile multiple"}

EPI_STORE, EPI_BIAS, EPI_BIAS_DROP_RESID, EPI_BIAS_RELU_DROP, EPI_RELU_DROP_BWD, EPI_ACCUM, EPI_ATTN_DS, \
    EPI_ATTN_DS_SIGNED, EPI_ATTN_DS_RECOMP, EPI_BIAS_DROP_RESID_LN, EPI_STORE_ROWDOT, EPI_STORE_ROWSTAT = range(12)
ABI_VERSION = 18   # include/u2gnn_hip.h U2GNN_ABI_VERSION
PREC_F32, PREC_BF16X3, PREC_BF16, PREC_BF16X6, PREC_F16X3 = 0, 1, 2, 3, 4


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("A", c_void_p), ("B", c_void_p), ("C", c_void_p),
        ("M", c_int64), ("N", c_int64), ("K", c_int64),
        ("lda", c_int64), ("ldb", c_int64), ("ldc", c_int64),
        ("trans_a", c_int32), ("trans_b", c_int32),
        ("epilogue", c_int32), ("split_k", c_int32),
        ("slab_stride", c_int64),
        ("bias", c_void_p), ("aux0", c_void_p), ("aux1", c_void_p), ("rowvec", c_void_p),
        ("ld_aux", c_int64),
        ("alpha", c_float),
        ("scale_cols", c_int64),
        ("p_drop", c_float),
        ("seed", c_uint64),
        ("precision", c_int32),
        ("tile", c_int32),
        ("keep", c_void_p), ("ld_keep", c_int64),
        ("clamp_a", c_int32), ("cx2_col0", c_int32),
        # ABI v3: pre-split (x2) operands / outputs
        ("a_x2", c_int32), ("b_x2", c_int32),
        ("A2", c_void_p), ("B2", c_void_p), ("Cx2", c_void_p), ("ldcx2", c_int64),
        ("rowstat", c_void_p), ("m_valid", c_int64), ("n_valid", c_int64),
        # ABI v7: LayerNorm fused into the bias-dropout-residual epilogue
        ("ln_gamma", c_void_p), ("ln_beta", c_void_p), ("ln_y", c_void_p), ("ln_ldy", c_int64),
        ("ln_mean", c_void_p), ("ln_rstd", c_void_p), ("ln_d", c_int64), ("ln_rows", c_int64),
        ("ln_eps", c_float), ("ln_reserved", c_int32),
        # ABI v8: delta = rowsum(dO * O) from the dO GEMM's epilogue (STORE_ROWDOT -> ATTN_DS_SIGNED)
        ("rowpart", c_void_p), ("ld_rowpart", c_int64),
        ("rowvec_parts", c_int32), ("rowvec_reserved", c_int32), ("ld_rowvec", c_int64),
        ("h3_exp_a", c_int32), ("h3_exp_b", c_int32),   # ABI v18: f16x3 operand pre-scales
    ]


class PackDesc(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("dst", c_void_p), ("ld_src", c_int64), ("rows_pad", c_int64),
                ("cols_pad", c_int64), ("rblk_pad", c_int64), ("rblk_real", c_int64), ("cblk_pad", c_int64),
                ("cblk_real", c_int64), ("ld_dst", c_int64)]


class ReduceJob(ctypes.Structure):   # u2gnn_reduce_job (ABI v11)
    _fields_ = [("kind", c_int32), ("n_slab", c_int32), ("accumulate", c_int32), ("alpha", c_float),
                ("src", c_void_p), ("ld_src", c_int64), ("slab_stride", c_int64), ("rows", c_int64),
                ("cols", c_int64), ("d", c_int64), ("rblk_pad", c_int64), ("rblk_real", c_int64),
                ("cblk_pad", c_int64), ("cblk_real", c_int64), ("dst", c_void_p), ("ld_dst", c_int64),
                ("Z", c_void_p), ("mean", c_void_p), ("rstd", c_void_p), ("dZdrop", c_void_p), ("ldz", c_int64),
                ("lddrop", c_int64), ("dbeta", c_void_p), ("dbias", c_void_p)]


RJOB_SLAB, RJOB_COLSUM, RJOB_LNPARAMS = 0, 1, 2


class LayerDims(ctypes.Structure):
    _fields_ = [("N", c_int64), ("d", c_int64), ("ff", c_int64), ("precision", c_int32), ("flags", c_int32),
                ("window", c_int32), ("reserved", c_int32)]


_PKEYS = ("in_w", "in_b", "out_w", "out_b", "l1_w", "l1_b", "l2_w", "l2_b", "n1_w", "n1_b", "n2_w", "n2_b")


class LayerParamsC(ctypes.Structure):
    _fields_ = [(k, c_void_p) for k in ("W_in", "b_in", "W_o", "b_o", "W1", "b1", "W2", "b2",
                                        "n1_w", "n1_b", "n2_w", "n2_b")]


class LayerSeeds(ctypes.Structure):
    _fields_ = [("p_drop", c_float), ("attn", c_uint64), ("drop1", c_uint64), ("dropff", c_uint64),
                ("drop2", c_uint64)]


class LayerGrads(ctypes.Structure):
    _fields_ = [(k, c_void_p) for k in _PKEYS]


_TAIL_PTRS = ("W_o", "b_o", "n1_w", "n1_b", "W1", "b1", "W2", "b2", "n2_w", "n2_b", "O", "X", "Z1", "X1", "mean1",
              "rstd1", "Hd", "Z2", "X2", "mean2", "rstd2", "dX2", "dX1", "dF", "dH", "dX", "dA", "dO", "delta")


class SmallTailArgs(ctypes.Structure):   # u2gnn_small_tail_args (ABI v15)
    _fields_ = ([(k, c_int64) for k in ("n_valid", "rows_pad", "d", "dp", "ff", "ffp")] +
                [("p", c_float), ("eps", c_float)] +
                [(k, c_uint64) for k in ("seed_drop1", "seed_dropff", "seed_drop2")] +
                [(k, c_void_p) for k in _TAIL_PTRS])


LAYER_DEEP_WGRAD = 1
LAYER_ATTN_BWD_BF16 = 2   # precision "mixed": dS, dQ, dK on plain bf16 (ABI v5)
LAYER_FWD_F32 = 4         # precision "fwd32": forward products exact fp32, backward bf16x3 (ABI v14)
LAYER_FWD_X6 = 8          # precision "fwd6": forward products bf16x6 (three-plane split), backward bf16x3 (ABI v17)
LAYER_FWD_H3 = 16         # precision "fwdh": forward products f16x3 (two-plane fp16 split), backward bf16x3 (ABI v18)
ROLE_QK, ROLE_PV, ROLE_DS, ROLE_DV, ROLE_DQ, ROLE_DK = range(1, 7)   # u2gnn_probe_arm roles

I64, F32, VP, I32 = c_int64, c_float, c_void_p, c_int32

_HIP_SIGS = {
    "u2gnn_abi_version": ([], c_int32),
    "u2gnn_gather_rows": ([VP, I64, I64, VP, I64, VP, I64, I64, I64, I64, I64, VP, VP], c_int32),
    "u2gnn_scatter_add_rows": ([VP, I64, VP, I64, VP, I64, I64, I64, I64, VP, VP], c_int32),
    "u2gnn_gemm": ([POINTER(GemmArgs), VP], c_int32),
    "u2gnn_gemm_group": ([POINTER(GemmArgs), I32, VP], c_int32),
    "u2gnn_reduce_batch_ws_floats": ([POINTER(ReduceJob), I32], I64),
    "u2gnn_reduce_batch": ([POINTER(ReduceJob), I32, VP, I64, VP], c_int32),
    "u2gnn_concat_dropout": ([POINTER(c_void_p), I32, I64, I64, I64, F32, c_uint64, VP, I64, VP], c_int32),
    "u2gnn_split_dropout_bwd": ([VP, I64, I32, I64, I64, I64, I64, F32, c_uint64, POINTER(c_void_p), VP], c_int32),
    "u2gnn_sum": ([VP, I64, VP, VP], c_int32),
    "u2gnn_sqnorm_partials": ([VP, I64, VP, VP], c_int32),
    "u2gnn_adam_sq": ([VP, VP, VP, VP, I64, VP, VP, F32, F32, F32, F32, F32, F32, VP], c_int32),
    "u2gnn_adam_dev_sq": ([VP, VP, VP, VP, I64, VP, VP, F32, c_double, c_double, F32, VP, VP, VP], c_int32),
    "u2gnn_layernorm_bwd_delta_slabs": ([VP, I64, VP, I32, I64, VP, I64, VP, VP, VP, VP, I64, VP, I64, F32, c_uint64,
                                         I64, I64, I64, I64, VP, I64, VP, VP, VP], c_int32),
    "u2gnn_slab_bias_drop_resid_ln": ([VP, I32, I64, I64, VP, VP, I64, F32, c_uint64, VP, I64, VP, VP, VP, I64, VP,
                                       VP, I64, I64, I64, F32, VP], c_int32),
    "u2gnn_index_zero_rows2": ([VP, I64, VP, I64, VP, I64, I64, I64, VP, VP], c_int32),
    "u2gnn_window_attn_fwd": ([VP, I64, I32, I32, VP, I64, VP, F32, c_uint64, I64, I64, VP], c_int32),
    "u2gnn_window_attn_bwd": ([VP, I64, I32, I32, VP, I64, VP, F32, c_uint64, F32, VP, I64, I64, I64, VP], c_int32),
    "u2gnn_layer_sizes": ([POINTER(LayerDims), F32, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)], c_int32),
    "u2gnn_layer_fwd": ([POINTER(LayerDims), POINTER(LayerParamsC), POINTER(LayerSeeds), VP, VP, VP, I64, VP, I64,
                         VP], c_int32),
    "u2gnn_layer_bwd": ([POINTER(LayerDims), POINTER(LayerParamsC), POINTER(LayerSeeds), VP, VP, I64, VP, VP,
                         POINTER(LayerGrads), VP, I64, VP, VP], c_int32),
    "u2gnn_slab_reduce": ([VP, I32, I64, I64, I64, I64, I64, I64, I64, I64, VP, I64, F32, I32, VP], c_int32),
    "u2gnn_pack_padded": ([VP, I64, I64, I64, I64, I64, I64, I64, VP, I64, VP], c_int32),
    "u2gnn_colsum": ([VP, I64, I64, I64, I64, I64, VP, I32, VP, VP], c_int32),
    "u2gnn_attn_softmax_fwd": ([VP, I64, VP, VP, I64, I64, I64, I64, I64, F32, c_uint64, VP, I64, VP], c_int32),
    "u2gnn_rowdot": ([VP, I64, VP, I64, VP, I64, I64, VP], c_int32),
    "u2gnn_split_x2": ([VP, I64, VP, I64, I64, I64, VP], c_int32),
    "u2gnn_layernorm_fwd": ([VP, I64, VP, VP, VP, I64, VP, VP, I64, I64, I64, I64, F32, VP], c_int32),
    "u2gnn_layernorm_bwd": ([VP, I64, VP, I64, VP, VP, VP, VP, I64, VP, I64, F32, c_uint64, I64, I64, I64, I64, VP],
                            c_int32),
    "u2gnn_layernorm_bwd_delta": ([VP, I64, VP, I64, VP, VP, VP, VP, I64, VP, I64, F32, c_uint64, I64, I64, I64, I64,
                                   VP, I64, VP, VP, VP], c_int32),
    "u2gnn_layernorm_bwd_params": ([VP, I64, VP, I64, VP, VP, VP, I64, I64, I64, I64, VP, VP, VP, VP, VP], c_int32),
    "u2gnn_pack_padded_multi": ([VP, I32, VP], c_int32),
    "u2gnn_pack_padded_multi_adv": ([VP, I32, VP, VP, VP], c_int32),
    "u2gnn_pool_fwd": ([VP, I64, VP, VP, VP, VP, I64, I64, I64, F32, c_uint64, VP], c_int32),
    "u2gnn_pool_bwd": ([VP, I64, VP, VP, VP, VP, I64, I64, I64, F32, c_uint64, VP], c_int32),
    "u2gnn_pool_bwd_rows": ([VP, I64, VP, VP, VP, VP, I64, I64, I64, I64, I64, I64, F32, c_uint64, VP], c_int32),
    "u2gnn_head_fwd": ([VP, I64, VP, VP, VP, I64, I64, I64, I32, VP], c_int32),
    "u2gnn_head_bwd": ([VP, VP, I64, VP, VP, I64, VP, VP, I64, I64, I64, I32, VP], c_int32),
    "u2gnn_smoothed_ce": ([VP, VP, I64, I64, F32, VP, VP, VP], c_int32),
    "u2gnn_sqnorm": ([VP, I64, VP, VP, VP], c_int32),
    "u2gnn_adam": ([VP, VP, VP, VP, I64, VP, F32, F32, F32, F32, F32, F32, VP], c_int32),
    "u2gnn_sampled_softmax_fwd": ([VP, I64, VP, VP, I64, VP, I64, VP, VP, I64, I64, VP], c_int32),
    "u2gnn_sampled_softmax_bwd": ([VP, I64, VP, VP, I64, VP, I64, VP, VP, VP, I64, VP, I64, I64, I64, VP], c_int32),
    "u2gnn_sampled_softmax_bwd_rows": ([VP, I64, VP, VP, I64, VP, I64, VP, VP, VP, I64, VP, I64, VP, I64, I64, I64, VP],
                                       c_int32),
    "u2gnn_index_add_rows": ([VP, I64, VP, I64, F32, VP, I64, I64, I64, VP, VP], c_int32),
    "u2gnn_index_zero_rows": ([VP, I64, VP, I64, I64, I64, VP, VP], c_int32),
    "u2gnn_dropout_mask": ([c_uint64, I64, I64, F32, VP, VP], c_int32),
    "u2gnn_dropout": ([VP, I64, VP, I64, I64, I64, F32, c_uint64, VP], c_int32),
    "u2gnn_attn_softmax_pv_ws_floats": ([I64, I64, I64], I64),
    "u2gnn_attn_softmax_pv": ([VP, I64, VP, I64, I64, VP, I64, I64, VP, I64, VP, I64, VP, I64, I64, I64, F32, c_uint64,
                               I32, VP],
                              c_int32),
    "u2gnn_attn_small_ctx_floats": ([I64, I64], I64),
    "u2gnn_layer_tail_small_fwd": ([ctypes.POINTER(SmallTailArgs), VP], c_int32),
    "u2gnn_layer_tail_small_bwd": ([ctypes.POINTER(SmallTailArgs), VP], c_int32),
    "u2gnn_layer_small_fwd": ([ctypes.POINTER(SmallTailArgs), VP, VP, c_uint64, VP, I64, VP], c_int32),
    "u2gnn_layer_small_bwd": ([ctypes.POINTER(SmallTailArgs), VP, c_uint64, VP, I64, VP, I64, I32, VP, I64, VP],
                              c_int32),
    "u2gnn_attn_small_ws_floats": ([I64, I64, I64], I64),
    "u2gnn_layer_tail_mid_ws_floats": ([I64, I64, I64], I64),
    "u2gnn_layer_tail_mid_fwd": ([ctypes.POINTER(SmallTailArgs), VP, I64, VP], c_int32),
    "u2gnn_attn_small_fwd": ([VP, I64, VP, VP, I64, I64, I64, I64, F32, c_uint64, VP, I64, VP, I64, VP], c_int32),
    "u2gnn_attn_small_bwd": ([VP, I64, VP, I64, I64, I64, I64, F32, c_uint64, VP, I64, VP, F32, VP, I64, VP, I64, VP,
                              I64, VP], c_int32),
    "u2gnn_probe_arm": ([I32, I32], c_int32),
    "u2gnn_probe_collect": ([POINTER(c_float), POINTER(c_int32)], c_int32),
    "u2gnn_set_seed_epoch": ([VP], c_int32),
    "u2gnn_step_advance": ([VP, VP, VP], c_int32),
    "u2gnn_adam_dev": ([VP, VP, VP, VP, I64, VP, F32, c_double, c_double, F32, VP, VP, VP], c_int32),
}

_LUS_SIGS = {
    "u2gnn_lus_create": ([I64, c_uint32], VP),
    "u2gnn_lus_destroy": ([VP], None),
    "u2gnn_lus_sample": ([VP, c_size_t, VP, POINTER(c_int32)], c_int32),
    "u2gnn_lus_sample_pyset": ([VP, c_size_t, VP, POINTER(c_int32)], c_int32),
    "u2gnn_lus_expected_count": ([VP, c_int32, VP, c_size_t, VP], c_int32),
    "u2gnn_lus_probability": ([VP, I64], c_float),
    "u2gnn_lus_sample_unique": ([VP, c_size_t, VP, c_size_t, VP], c_int32),
    "u2gnn_lus_accidental_matches": ([VP, c_size_t, VP, c_size_t, VP, c_size_t, POINTER(c_size_t)], c_int32),
    "u2gnn_batch_assemble": ([VP, POINTER(c_int32), VP, I64, VP, VP, VP, VP, VP, I32, I64, VP, VP, VP], c_int32),
}

_hip = None
_lus = None


def _bind(lib, sigs):
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def hip_lib():
    """The gfx950 kernel library; raises if it is not built (no CPU fallback exists)."""
    global _hip
    if _hip is None:
        if not os.path.exists(HIP_LIB_PATH):
            raise U2GNNNativeError(f"{HIP_LIB_PATH} not built: run `make -C graph-transformer_amd/csrc` "
                                   "(the U2GNN hot path has no CPU fallback)")
        try:
            lib = ctypes.CDLL(HIP_LIB_PATH)
        except OSError as e:  # pragma: no cover
            raise U2GNNNativeError(f"cannot load {HIP_LIB_PATH}: {e}") from e
        _hip = _bind(lib, _HIP_SIGS)
        v = _hip.u2gnn_abi_version()
        if v != ABI_VERSION:
            raise U2GNNNativeError(f"ABI mismatch: library {v}, binding {ABI_VERSION}")
    return _hip




def lus_lib():
    global _lus
    if _lus is None:
        if not os.path.exists(LUS_LIB_PATH):
            raise U2GNNNativeError(f"{LUS_LIB_PATH} not built: run `make -C graph-transformer_amd/csrc`")
        _lus = _bind(ctypes.CDLL(LUS_LIB_PATH), _LUS_SIGS)
    return _lus


def check(rc: int, what: str):
    if rc != 0:
        msg = ERRORS.get(rc, f"hipError {rc}")
        raise U2GNNNativeError(f"{what} failed: {msg} (rc={rc})")


def source_build_id() -> str:
    """Hash of the native sources (csrc/ + include/): the build a profile was taken from.  bench.py
    uses a committed PMC traffic table only when its recorded build id equals this one."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(PKG_ROOT, "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile")
    files += sorted(os.path.join(INCLUDE_DIR, f) for f in os.listdir(INCLUDE_DIR) if f.endswith(".h"))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def header_symbols(header: str):
    """Function names declared in include/<header> (used by the ABI export test)."""
    txt = open(os.path.join(INCLUDE_DIR, header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(u2gnn_[a-z0-9_]+)\s*\(", txt)))
