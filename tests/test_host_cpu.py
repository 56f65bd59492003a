"""Host-side product code on CPU: the C-ABI libraries load and export every declared symbol,
the native sampler equals the reference's, the loader equals the networkx-based oracle loader,
and the vectorised batch assembly is bit-exact with the reference's per-node loop."""
import os

import numpy as np
import pytest
import torch

from oracle import u2gnn_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(REPO, "dataset")


# ------------------------------------------------------------------------------- C ABI
@pytest.mark.parametrize("header,loader", [("u2gnn_hip.h", "hip_lib"), ("u2gnn_lus.h", "lus_lib")])
def test_libraries_export_every_header_symbol(header, loader):
    from u2gnn_hip import _lib
    lib = getattr(_lib, loader)()
    syms = _lib.header_symbols(header)
    assert len(syms) >= 7
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    if loader == "hip_lib":
        assert lib.u2gnn_abi_version() == _lib.ABI_VERSION == 18


def test_kernel_wrappers_refuse_host_tensors():
    from u2gnn_hip import U2GNNNativeError
    from u2gnn_hip import kernels as K
    x = torch.zeros(4, 4)
    with pytest.raises(U2GNNNativeError):
        K.gemm(x, x, x, 4, 4, 4, 4, 4, 4)


def test_gemm_argument_validation_without_gpu():
    """Shape/alignment checks run on the host before any launch."""
    import ctypes
    from u2gnn_hip import _lib
    lib = _lib.hip_lib()
    a = _lib.GemmArgs()
    assert lib.u2gnn_gemm(ctypes.byref(a), None) == -1          # null pointers
    a.A = a.B = a.C = 16
    a.M, a.N, a.K, a.lda, a.ldb = 64, 64, 24, 24, 64
    assert lib.u2gnn_gemm(ctypes.byref(a), None) == -3          # K not a multiple of 16
    a.K, a.lda = 32, 30
    assert lib.u2gnn_gemm(ctypes.byref(a), None) == -2          # lda not 16-byte aligned
    a.lda, a.precision = 32, 7
    assert lib.u2gnn_gemm(ctypes.byref(a), None) == -1          # unknown precision


# ------------------------------------------------------------------------------- sampler
def test_native_sampler_equals_reference_order_and_counts(golden_dir):
    from log_uniform import LogUniformSampler
    z = dict(np.load(os.path.join(golden_dir, "sampler.npz")))
    for V in (8792, 2542091):
        s = LogUniformSampler(V)
        for c in range(3):
            ids, tf, sf = s.sample(512, np.arange(4, dtype=np.int64))
            assert ids == z[f"V{V}_c{c}_ids_order"].tolist()            # same unordered_set order
            assert np.array_equal(np.asarray(sf, np.float32), z[f"V{V}_c{c}_sample_freq"])
            assert np.array_equal(np.asarray(tf, np.float32), z[f"V{V}_c{c}_true_freq"])


def test_native_sampler_edge_cases():
    from log_uniform import LogUniformSampler
    s = LogUniformSampler(10)
    ids, _ = s.sample_ids(10)                  # size == N terminates with every id
    assert sorted(ids.tolist()) == list(range(10))
    with pytest.raises(ValueError):            # the reference would loop forever
        s.sample_ids(11)
    u = s.sample_unique(5, [0, 1, 2])
    assert len(set(u)) == 5 and not set(u) & {0, 1, 2}
    with pytest.raises(ValueError):
        s.sample_unique(8, [0, 1, 2])
    assert s.accidental_match([3, 9, 4], [4, 3, 7]) == [(0, 1), (2, 0)]
    p = np.array([s.probability(i) for i in range(10)])
    assert abs(p.sum() - 1.0) < 1e-6 and np.all(np.diff(p) < 0)


# ------------------------------------------------------------------------------- loader
@pytest.mark.parametrize("name,deg", [("MUTAG", False), ("PTC", False), ("IMDBBINARY", True)])
def test_loader_equals_networkx_oracle(name, deg):
    import util
    ours, c1 = util.load_data(name, deg)
    ref, c2 = O.load_data(os.path.join(DATA, name, name + ".txt"), deg)
    assert c1 == c2 and len(ours) == len(ref)
    for a, b in zip(ours, ref):
        assert a.label == b.label and a.n == b.n
        assert np.array_equal(a.edge_mat, b.edge_mat)
        assert np.array_equal(a.node_features, b.node_features)


def test_split_is_stratified_and_fixed():
    import util
    graphs, _ = util.load_data("MUTAG", False)
    tr, te = util.separate_data_idx(graphs, 1)
    z = dict(np.load(os.path.join(REPO, "tests", "golden", "mutag_sup.npz")))
    assert np.array_equal(tr, z["train_idx"]) and np.array_equal(te, z["test_idx"])


# ------------------------------------------------------------------------------- batches
@pytest.mark.parametrize("name,deg,k", [("MUTAG", False, 4), ("IMDBBINARY", True, 8), ("PTC", False, 16)])
def test_vectorised_batches_bit_exact(name, deg, k):
    import util
    from u2gnn_hip.batching import BatchLoader, GraphStore
    graphs, _ = util.load_data(name, deg)
    ref_graphs, _ = O.load_data(os.path.join(DATA, name, name + ".txt"), deg)
    store = GraphStore(graphs)
    np.random.seed(123)
    bl = BatchLoader(store, 32, k)
    ours = [bl() for _ in range(4)]
    tail_ours = np.random.randint(0, 1 << 30, 4)
    np.random.seed(123)
    for b in ours:
        sel = np.random.permutation(len(ref_graphs))[:32]
        ix, off, X, y = O.get_batch_data_seq([ref_graphs[i] for i in sel], k)
        assert np.array_equal(b.graph_ids, sel)
        assert np.array_equal(b.input_x, ix) and np.array_equal(b.offsets, off)
        assert np.array_equal(b.X_concat, X) and np.array_equal(b.labels, y)
    assert np.array_equal(np.random.randint(0, 1 << 30, 4), tail_ours)     # stream left aligned


def test_golden_batches_reproduced_by_product_loader(golden_dir):
    """The seed-123 stream over the fold-1 train split gives the fixtures' input_x."""
    import util
    from u2gnn_hip.batching import BatchLoader, GraphStore
    z = dict(np.load(os.path.join(golden_dir, "imdbb_sup.npz")))
    graphs, _ = util.load_data("IMDBBINARY", True)
    train, _ = util.separate_data(graphs, 1)
    np.random.seed(123)
    bl = BatchLoader(GraphStore(train), 4, 8)
    for i in range(3):
        b = bl()
        assert np.array_equal(b.input_x, z[f"b{i}_input_x"]) and np.array_equal(b.X_concat, z[f"b{i}_X"])


def test_replay_consumes_the_same_stream():
    import util
    from u2gnn_hip.batching import BatchLoader, GraphStore
    graphs, _ = util.load_data("PTC", False)
    store = GraphStore(graphs)
    np.random.seed(5)
    bl = BatchLoader(store, 8, 4)
    full = [bl() for _ in range(3)]
    np.random.seed(5)
    bl.replay()
    b1 = bl()
    bl.replay()
    assert np.array_equal(b1.input_x, full[1].input_x)
    np.random.seed(5)
    for _ in range(3):
        bl()
    a = np.random.rand()
    np.random.seed(5)
    for _ in range(3):
        bl.replay()
    assert np.random.rand() == a


def test_synthetic_collab_statistics():
    from u2gnn_hip.synthetic import collab_like
    s = collab_like()
    assert len(s.graphs) == 5000 and abs(s.n_nodes.mean() - 74.49) < 0.5
    assert s.n_nodes.min() >= 32 and s.n_nodes.max() <= 492
    np.random.seed(0)
    b = s.assemble(np.arange(20), 16)
    e = sum(len(s.graph(i)[1]) for i in range(200)) / 2 / 200
    assert 1800 < e < 3200                         # ~2457.78 edges per graph
    assert b.input_x.shape[1] == 17 and b.X_concat.shape[1] == 367
    # every sampled neighbour is a real neighbour inside the same graph
    off = b.offsets
    for g in range(20):
        rows = b.input_x[off[g]:off[g + 1]]
        assert rows.min() >= off[g] and rows.max() < off[g + 1]


def test_native_assembly_equals_numpy_form_and_stream():
    """csrc/batch_assembly.cpp continues numpy's MT19937 stream exactly like the numpy randint form:
    same input_x / offsets / X and the same generator state afterwards (isolated nodes, degree 1,
    degrees past 2^16 so that the rejection mask spans 17 bits, k = 0)."""
    from u2gnn_hip.batching import GraphStore

    class G:
        def __init__(self, n, src, dst, label):
            self.n, self.label = n, label
            self.edge_mat = np.stack([src, dst]).astype(np.int64)
            self.node_features = np.eye(5, dtype=np.float32)[np.arange(n) % 5]

    rs = np.random.RandomState(7)
    graphs = []
    for gi in range(40):
        n = int(rs.randint(1, 60))
        m = int(rs.randint(0, 4 * n))
        src, dst = rs.randint(0, n, m), rs.randint(0, n, m)
        graphs.append(G(n, np.concatenate([src, dst]), np.concatenate([dst, src]), gi % 3))
    hub = 70000                                   # one node with 70000 (multi-)edges
    graphs.append(G(3, np.concatenate([np.zeros(hub, np.int64), [1]]), np.concatenate([np.ones(hub, np.int64), [0]]),
                    1))
    store = GraphStore(graphs)
    for k in (0, 1, 16):
        for seed in (0, 1):
            np.random.seed(seed)
            ref = []
            for _ in range(5):
                sel = np.random.permutation(len(graphs))[:12]
                ref.append(store.assemble_numpy(sel, k))
            st_ref = np.random.get_state()
            np.random.seed(seed)
            for r in ref:
                sel = np.random.permutation(len(graphs))[:12]
                b = store.assemble(sel, k)
                assert np.array_equal(b.input_x, r.input_x) and np.array_equal(b.offsets, r.offsets)
                assert np.array_equal(b.X_concat, r.X_concat) and np.array_equal(b.labels, r.labels)
            st = np.random.get_state()
            assert np.array_equal(st[1], st_ref[1]) and st[2] == st_ref[2]
    np.random.seed(3)                             # a batch holding the hub node
    a = store.assemble([40, 2], 16)
    np.random.seed(3)
    b = store.assemble_numpy([40, 2], 16)
    assert np.array_equal(a.input_x, b.input_x)


def test_device_batch_rejects_out_of_range_input_x():
    """F.embedding(input_x, X_concat) raises IndexError for an entry outside [0, N)
    (pytorch_U2GNN_Sup.py:32); the batch constructors check before anything reaches a kernel."""
    import numpy as np
    from u2gnn_hip.core import DeviceBatch
    X = np.zeros((5, 3), np.float32)
    off = np.array([0, 2, 5])
    for bad in (5, -1):
        ix = np.tile(np.arange(5)[:, None], (1, 3))
        ix[4, 2] = bad
        with pytest.raises(IndexError):
            DeviceBatch.from_offsets(ix, off, X, np.array([0, 1]), device="cpu")


def test_layer_executor_refuses_undersized_buffers_before_launching():
    """u2gnn_layer_fwd / u2gnn_layer_bwd plan the call first and refuse a workspace or ctx arena smaller than
    it takes (U2GNN_E_ARG) before any launch: on this GPU-less host a launch would fail with a HIP error
    code instead, so -1 shows that nothing was launched (no kernel can write past a caller buffer)."""
    import ctypes
    from u2gnn_hip import _lib
    lib = _lib.hip_lib()
    dims = _lib.LayerDims(1914, 4, 1024, 1, 0, 0, 0)   # the C5 layer, bf16x3
    c, f, b = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    assert lib.u2gnn_layer_sizes(ctypes.byref(dims), 0.5, ctypes.byref(c), ctypes.byref(f), ctypes.byref(b)) == 0
    fake = ctypes.c_void_p(1 << 40)   # never dereferenced on the host
    params = _lib.LayerParamsC(*([fake.value] * 12))
    seeds = _lib.LayerSeeds(0.5, 1, 2, 3, 4)
    grads = _lib.LayerGrads(*([fake.value] * len(_lib._PKEYS)))
    rc = lib.u2gnn_layer_fwd(ctypes.byref(dims), ctypes.byref(params), ctypes.byref(seeds), fake, fake, fake, c.value,
                             fake, f.value - 256, None)
    assert rc == -1
    rc = lib.u2gnn_layer_bwd(ctypes.byref(dims), ctypes.byref(params), ctypes.byref(seeds), fake, fake, c.value, fake,
                             fake, ctypes.byref(grads), fake, b.value - 256, None, None)
    assert rc == -1
    rc = lib.u2gnn_layer_bwd(ctypes.byref(dims), ctypes.byref(params), ctypes.byref(seeds), fake, fake, c.value - 256,
                             fake, fake, ctypes.byref(grads), fake, b.value, None, None)
    assert rc == -1


def test_round5_shape_rules():
    """The Python orchestration's copies of the executor's round-5 shape rules (encoder_layer.cpp mid_tail,
    ffn2_split; engine.py mirrors them launch for launch) at the bench configurations, and the mid tail's
    workspace sizing (a host-only entry point)."""
    from u2gnn_hip import engine as E
    from u2gnn_hip import kernels as K
    assert E.mid_tail(136, 192, 128) and E.mid_tail(100, 128, 128) and E.mid_tail(40, 64, 512)   # C2-class
    assert not E.mid_tail(32, 64, 128)        # d <= 32: the small-width layer
    assert not E.mid_tail(367, 384, 4864)     # C4: the matrix-core path
    assert not E.mid_tail(136, 192, 640)      # more than 512 padded rows
    assert E.ffn2_split(128, True, 128, 1024) == 8     # C2: 4 output tiles -> 8 slabs of 4 K steps
    assert E.ffn2_split(384, True, 4864, 1024) == 1    # C4: 456 tiles fill the chip
    assert E.ffn2_split(64, True, 2048, 1024) == 8     # a d <= 64 layer at 2048 rows (the round-3 rule)
    assert E.ffn2_split(128, False, 128, 1024) == 1    # fp32 parity path: no split
    assert E.ffn2_split(320, True, 128, 1024) == 1     # dp > 256: no slab LayerNorm
    assert K.layer_tail_mid_ws_floats(128, 128, 1024) == 8 * 128 * 128
    assert K.layer_tail_mid_ws_floats(128, 192, 256) == 2 * 128 * 192   # ff = 200 padded to 256: 2 chunks
    assert K.layer_tail_mid_ws_floats(128, 192, 200) == -1              # unpadded widths are refused
    assert K.layer_tail_mid_ws_floats(128, 320, 1024) == -1
