import functools
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "privileged: needs root + a real cgroup/bpf kernel "
                                       "(run when the host allows it; GM_PRIVILEGED_TESTS=0/1 "
                                       "forces off/on)")


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


@functools.lru_cache(maxsize=None)
def privileged_ok() -> bool:
    """Whether the privileged real-kernel tests run here. GM_PRIVILEGED_TESTS=1 forces them on,
    =0 off; otherwise they run when this process is root and the kernel lets it mount a private
    cgroup2 hierarchy and load a device BPF program (the development container does; the
    unprivileged GPU box does not, and they are skipped there)."""
    env = os.environ.get("GM_PRIVILEGED_TESTS", "")
    if env == "0" or os.geteuid() != 0:
        return False
    if env == "1":
        return True
    try:
        r = subprocess.run(["unshare", "-m", "--propagation", "private", "sh", "-c",
                            'd=$(mktemp -d) && mount -t cgroup2 none "$d" && umount "$d" && '
                            'rmdir "$d"'], capture_output=True, timeout=30)
        if r.returncode != 0:
            return False
        import ctypes as C

        from gpumounter_amd import _native
        lib = _native.host()
        rules = (_native.DevRule * 1)(_native.DevRule(b"c", 7, 1, 0, 1, 3))
        need = -lib.gm_bpf_dev_build(rules, 1, 0, -1, None, 0)
        buf = (C.c_uint64 * need)()
        n = lib.gm_bpf_dev_build(rules, 1, 0, -1, buf, need)
        fd = lib.gm_bpf_dev_load(buf, n, b"gm_probe", None, 0)
        if fd < 0:
            return False
        os.close(fd)
        return True
    except Exception:  # noqa: BLE001 - any failure means: not here
        return False


def privileged_skip():
    return pytest.mark.skipif(not privileged_ok(),
                              reason="privileged real-kernel test: needs root with mount + bpf "
                                     "(GM_PRIVILEGED_TESTS=1 forces it)")
