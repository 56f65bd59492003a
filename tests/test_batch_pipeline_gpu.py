"""Native batch assembly + GPU feature gather (DeviceBatch.from_store) against the host path
(DeviceBatch.from_offsets of the numpy-form batch): identical device tensors, bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,deg,k", [("MUTAG", False, 4), ("IMDBBINARY", True, 8)])
def test_from_store_equals_host_path(name, deg, k):
    import util
    from u2gnn_hip.batching import BatchLoader, GraphStore
    from u2gnn_hip.core import DeviceBatch
    graphs, _ = util.load_data(name, deg)
    store = GraphStore(graphs)
    X_dev = torch.from_numpy(store.X).cuda()
    np.random.seed(11)
    ref = [BatchLoader(store, 32, k, native=False, with_input_y=True)() for _ in range(3)]
    np.random.seed(11)
    loader = BatchLoader(store, 32, k, gather_x=False, with_input_y=True)
    for r in ref:
        a = DeviceBatch.from_store(loader(), X_dev)
        b = DeviceBatch.from_offsets(r.input_x, r.offsets, r.X_concat, r.labels, input_y=r.input_y)
        torch.cuda.synchronize()
        assert a.N == b.N and a.B == b.B
        for f in ("input_x", "X_concat", "rowptr", "colidx", "vals", "labels", "input_y"):
            assert torch.equal(getattr(a, f), getattr(b, f)), f
