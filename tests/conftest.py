import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu_device():
    """The product path has no CPU fallback: a GPU test without a GPU fails loudly."""
    from crdt_amd import _capi
    n = _capi.device_count()
    assert n > 0, "no gfx950 device visible: GPU tests need an MI355X"
    return 0


@pytest.fixture(autouse=True)
def _fixed_routing(monkeypatch):
    """Sharded fan-ins take the fixed routing rule in tests (each way is asserted explicitly); the routing
    tuner, which picks a way per ctx from measured calls, has its own test (test_two_rank_route_tune)."""
    monkeypatch.setenv("CRDT_ROUTE_TUNE", "0")
