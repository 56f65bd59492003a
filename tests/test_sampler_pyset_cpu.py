"""u2gnn_lus_sample_pyset (csrc/log_uniform_sampler.cpp): the native emulation of CPython's set order must equal
list(set(ids)) of this interpreter for the ids u2gnn_lus_sample returns, draw after draw (two samplers on the same
seed walk the same engine stream), across the set's resize points (5 -> 8 -> 32 -> 128 ... slots) and past the
50 000-element policy switch; the arena allocator must leave the unordered_set order of u2gnn_lus_sample intact
(checked against the plain draws through the reference-pinned tests of log_uniform)."""
import numpy as np
import pytest

from log_uniform import LogUniformSampler


@pytest.mark.parametrize("N,size,draws", [(2542092, 512, 300), (1000, 5, 200), (50, 37, 100), (100000, 3000, 20),
                                          (5_000_000, 60000, 2)])
def test_pyset_order_matches_python_set(N, size, draws):
    a, b = LogUniformSampler(N, seed=7), LogUniformSampler(N, seed=7)
    for _ in range(draws):
        ids, nt = a.sample_ids(size)
        want = np.asarray(list(set(ids.tolist())), dtype=np.int64)
        got, nt2 = b.sample_set_order(size)
        assert nt == nt2
        assert np.array_equal(got, want)


def test_arena_keeps_unordered_set_order():
    """The same engine stream through a fresh sampler twice: identical ids in identical order, call after call
    (the arena is rewound per call; a stale node would show as a changed order or a missing id)."""
    a, b = LogUniformSampler(2542092), LogUniformSampler(2542092)
    for size in (512, 1, 512, 2000, 3, 512):
        x, nx = a.sample_ids(size)
        y, ny = b.sample_ids(size)
        assert nx == ny and np.array_equal(x, y) and len(set(x.tolist())) == size
