import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "privileged: needs root + a real cgroup/bpf kernel "
                                       "(opt-in: GM_PRIVILEGED_TESTS=1)")


@pytest.fixture(scope="session", autouse=True)
def _native_libs():
    from gpumounter_amd import _native

    _native.host()
    _native.smi()
    yield
    _native.record_maps()          # GM_RECORD_MAPS=<file>: which in-tree .so files were mapped


@pytest.fixture(scope="session")
def mock_inventory():
    """Process-wide amdsmi session on the bundled mock (8×MI355X, one hive, 2 NUMA nodes)."""
    from gpumounter_amd.hw.inventory import Inventory

    return Inventory("mock")


def has_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False
