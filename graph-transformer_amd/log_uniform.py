"""Drop-in replacement of the reference's Cython module ``log_uniform`` (log_uniform.pyx:16-40)
over the native sampler libu2gnn_lus.so (C ABI: include/u2gnn_lus.h).

Same class, constructor and method names/returns; the engine, distribution and set semantics
are the reference's, so ``sample`` returns the same ids in the same (unordered_set) order.
"""
import ctypes

import numpy as np

from u2gnn_hip._lib import U2GNNNativeError, lus_lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


class LogUniformSampler(object):
    def __init__(self, N, seed=1111):
        self.N = int(N)
        self._lib = lus_lib()
        self._h = self._lib.u2gnn_lus_create(self.N, int(seed))
        if not self._h:
            raise U2GNNNativeError("u2gnn_lus_create failed")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.u2gnn_lus_destroy(h)

    def sample_ids(self, size):
        """Fast path: (int64 ndarray of `size` ids, num_tries)."""
        out = np.empty(int(size), dtype=np.int64)
        nt = ctypes.c_int32()
        rc = self._lib.u2gnn_lus_sample(self._h, int(size), _ptr(out), ctypes.byref(nt))
        if rc != 0:
            raise ValueError(f"sample({size}) rejected (N={self.N}); the reference would not terminate"
                             if rc == -1 else f"sampler error {rc}")
        return out, nt.value

    def expected_count(self, num_tries, ids):
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int64).reshape(-1))
        out = np.empty(ids.size, dtype=np.float32)
        rc = self._lib.u2gnn_lus_expected_count(self._h, int(num_tries), _ptr(ids), ids.size, _ptr(out))
        if rc != 0:
            raise IndexError("id out of range")
        return out

    def sample_set_order(self, size):
        """ids in the order the reference returns them: its Cython binding converts the C++
        unordered_set into a Python set (inserting in C++ iteration order) before list() -- that
        set order computed natively (u2gnn_lus_sample_pyset; equal to list(set(sample_ids order)),
        tests/test_sampler_pyset_cpu.py)."""
        out = np.empty(int(size), dtype=np.int64)
        nt = ctypes.c_int32()
        rc = self._lib.u2gnn_lus_sample_pyset(self._h, int(size), _ptr(out), ctypes.byref(nt))
        if rc != 0:
            raise ValueError(f"sample({size}) rejected (N={self.N}); the reference would not terminate"
                             if rc == -1 else f"sampler error {rc}")
        return out, nt.value

    def sample(self, size, labels):
        """log_uniform.pyx:29-34: (sample ids, true expected counts, sample expected counts)."""
        ids, nt = self.sample_set_order(size)
        true_freq = self.expected_count(nt, np.asarray(labels)).tolist()
        sample_freq = self.expected_count(nt, ids).tolist()
        return ids.tolist(), true_freq, sample_freq

    def sample_unique(self, size, labels):
        ex = np.ascontiguousarray(np.asarray(list(labels), dtype=np.int64).reshape(-1))
        out = np.empty(int(size), dtype=np.int64)
        rc = self._lib.u2gnn_lus_sample_unique(self._h, int(size), _ptr(ex), ex.size, _ptr(out))
        if rc != 0:
            raise ValueError("sample_unique rejected: size exceeds the ids left after exclusion")
        return out.tolist()

    def accidental_match(self, labels, samples):
        la = np.ascontiguousarray(np.asarray(labels, dtype=np.int64).reshape(-1))
        sa = np.ascontiguousarray(np.asarray(samples, dtype=np.int64).reshape(-1))
        out = np.empty(2 * max(1, la.size), dtype=np.int64)
        n = ctypes.c_size_t()
        rc = self._lib.u2gnn_lus_accidental_matches(_ptr(la), la.size, _ptr(sa), sa.size, _ptr(out), la.size,
                                                    ctypes.byref(n))
        if rc != 0:
            raise RuntimeError("accidental_matches failed")
        return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n.value)]

    def probability(self, idx):
        return float(self._lib.u2gnn_lus_probability(self._h, int(idx)))
