import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "graph-transformer_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def rdzv_port():
    """Rendezvous for a multi-process test: a TCPStore bound HERE on a port the kernel picks and held open for the
    test, so no other process can take it between a probe and the workers' connect (the probe-then-close race).
    Workers reach it as clients: MASTER_ADDR=127.0.0.1, MASTER_PORT=<this port>, TORCHELASTIC_USE_AGENT_STORE=True
    (torch.distributed's env:// then makes every rank a client of an existing store, as under torchrun).  One
    process group per store: a fixture per test."""
    from torch.distributed import TCPStore
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False)
    yield store.port
    del store
