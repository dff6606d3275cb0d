import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _close_distributed_runtimes():
    """Every DistributedMooseRuntime a test made is closed after it (their worker pools
    would otherwise run until the test process exits)."""
    yield
    try:
        from moose_amd.runtime import distributed
    except Exception:  # noqa: BLE001
        return
    for rt in list(distributed._LIVE):
        try:
            rt.close()
        except Exception:  # noqa: BLE001
            pass
