"""Host natives under AddressSanitizer + UBSan:
csrc/batch_assembly.cpp and csrc/log_uniform_sampler.cpp do raw index arithmetic over caller arrays
(the CSR, nbr_start, the MT state).  tests/asan/host_asan_driver.cpp links them with
-fsanitize=address,undefined into a standalone program (no Python in the instrumented process), runs
the assembly over random graphs, a 70 000-edge hub (17-bit rejection masks), isolated nodes, k = 0 / 1
/ 16, MUTAG batches and a too-small output capacity, and the sampler over V = 8792 / 2.54 M, size > N
and sample_unique / accidental_matches; every output must equal the regular build's."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "graph-transformer_amd", "csrc")


def _build(tmp):
    exe = os.path.join(tmp, "host_asan_driver")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-static-libasan", "-static-libubsan", "-I", os.path.join(REPO, "include"),
           "-o", exe, os.path.join(REPO, "tests", "asan", "host_asan_driver.cpp"),
           os.path.join(CSRC, "batch_assembly.cpp"), os.path.join(CSRC, "log_uniform_sampler.cpp")]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe


class _G:
    def __init__(self, n, src, dst, label):
        self.n, self.label = n, label
        self.edge_mat = np.stack([src, dst]).astype(np.int64)
        self.node_features = np.eye(5, dtype=np.float32)[np.arange(n) % 5]


def _stores():
    import util
    from u2gnn_hip.batching import GraphStore
    rs = np.random.RandomState(7)
    graphs = []
    for gi in range(40):
        n = int(rs.randint(1, 60))
        m = int(rs.randint(0, 4 * n))
        src, dst = rs.randint(0, n, m), rs.randint(0, n, m)
        graphs.append(_G(n, np.concatenate([src, dst]), np.concatenate([dst, src]), gi % 3))
    hub = 70000
    graphs.append(_G(3, np.concatenate([np.zeros(hub, np.int64), [1]]), np.concatenate([np.ones(hub, np.int64), [0]]), 1))
    mutag, _ = util.load_data("MUTAG", False)
    return [GraphStore(graphs), GraphStore(mutag)]


def test_host_natives_under_asan(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    from u2gnn_hip._lib import lus_lib
    exe = _build(str(tmp_path))
    recs, expect = [], []
    n_asm = 0
    for si, store in enumerate(_stores()):
        for k in (0, 1, 16):
            for seed in (0, 5):
                np.random.seed(seed + 10 * si)
                sel = np.random.permutation(len(store.graphs))[:12]
                if si == 0:
                    sel = np.concatenate([[40], sel[:11]])   # always hold the hub graph
                st = np.random.get_state()
                N = int(store.n_nodes[sel].sum())
                for cap in (N, N - 1):                       # N - 1: rejected, nothing written
                    recs.append([np.asarray(st[1], np.int64), [int(st[2])], [len(sel)], sel, [len(store.n_nodes)],
                                 store.n_nodes, store.node_start, [len(store.deg)], store.deg, store.nbr_start,
                                 [len(store.nbr)], store.nbr, [k], [max(cap, 0)]])
                    n_asm += 1
                    if cap == N:
                        np.random.set_state(st)
                        b = store.assemble(sel, k, gather_x=False)
                        st2 = np.random.get_state()
                        expect.append((0, b.offsets, b.input_x.ravel(), b.gnode, np.asarray(st2[1], np.int64), st2[2]))
                    else:
                        expect.append((-1, None, None, None, np.asarray(st[1], np.int64), st[2]))
    lus_cases = [(8792, 1111, 512, 3, [0, 5, 17]), (2542091, 1111, 512, 2, [1, 2, 3, 100]), (100, 1111, 200, 1, [1]),
                 (64, 7, 60, 2, list(range(10)))]
    with open(os.path.join(tmp_path, "in.bin"), "wb") as f:
        np.asarray([n_asm, len(lus_cases)], np.int64).tofile(f)
        for r in recs:
            for a in r:
                np.asarray(a, np.int64).tofile(f)
        for (N, seed, size, reps, excl) in lus_cases:
            np.asarray([N, seed, size, reps, len(excl)] + excl, np.int64).tofile(f)
    p = subprocess.run([exe, os.path.join(tmp_path, "in.bin"), os.path.join(tmp_path, "out.bin")], capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    out = np.fromfile(os.path.join(tmp_path, "out.bin"), dtype=np.int64)
    pos = [0]

    def get():
        pos[0] += 1
        return int(out[pos[0] - 1])

    def vec():
        n = get()
        v = out[pos[0]:pos[0] + n]
        pos[0] += n
        return v
    for rc, off, ix, gn, key, mtpos in expect:
        assert get() == rc
        o, x, g = vec(), vec(), vec()
        if rc == 0:
            assert np.array_equal(o, off) and np.array_equal(x, ix) and np.array_equal(g, gn)
        assert np.array_equal(vec(), key) and get() == mtpos
    lib = lus_lib()
    for (N, seed, size, reps, excl) in lus_cases:
        h = lib.u2gnn_lus_create(N, seed)
        ids = np.zeros(size, np.int64)
        ec = np.zeros(size, np.float32)
        P = lambda a: a.ctypes.data  # noqa: E731
        for _ in range(reps):
            tries = ctypes.c_int32(0)
            rc = lib.u2gnn_lus_sample(h, size, P(ids), ctypes.byref(tries))
            assert get() == rc and get() == tries.value
            got = vec()
            if rc == 0:
                assert np.array_equal(got, ids)
            rc2 = lib.u2gnn_lus_expected_count(h, tries.value, P(ids), size, P(ec)) if rc == 0 else -1
            assert get() == rc2
            got = vec()
            if rc2 == 0:
                assert np.array_equal(got.astype(np.uint32).view(np.float32), ec)
        ex = np.asarray(excl, np.int64)
        rc3 = lib.u2gnn_lus_sample_unique(h, size, P(ex), len(ex), P(ids))
        assert get() == rc3
        got = vec()
        if rc3 == 0:
            assert np.array_equal(got, ids) and not set(ids.tolist()) & set(excl)
        pairs = np.zeros(2 * len(ex) * size + 2, np.int64)
        n_out = ctypes.c_size_t(0)
        rc4 = lib.u2gnn_lus_accidental_matches(P(ex), len(ex), P(ids), size if rc3 == 0 else 0, P(pairs),
                                               len(ex) * size + 1, ctypes.byref(n_out))
        assert get() == rc4
        got = vec()
        if rc4 == 0:
            assert np.array_equal(got, pairs[:2 * n_out.value])
        lib.u2gnn_lus_destroy(h)
    assert pos[0] == len(out)
