"""GPU busy detection and process termination.

Reference: busy ⇔ some NVML graphics/compute PID of the GPU is in the container's
``cgroup.procs`` (reference: pkg/util/util.go:152-196), with NVML re-initialised per query
(pkg/device/nvidia.go:58-87), and force-removal runs ``kill <pids>`` through nsenter
(namespace.go:191-201). Here the PID set comes from the cached amdsmi session
(``amdsmi_get_gpu_process_list``), with a ``/proc/*/fd`` scan for the GPU's render node as
fallback when amdsmi cannot report processes; signals go through ``pidfd_send_signal`` so a
recycled PID is never hit, and SIGTERM escalates to SIGKILL after a grace period.
"""
from __future__ import annotations

import asyncio
import ctypes as C
import os
import signal
from typing import Dict, Iterable, List, Sequence

from gpumounter_amd import _native
from gpumounter_amd.hw.inventory import Inventory
from gpumounter_amd.models.device import DRM_MAJOR, AmdGpu
from gpumounter_amd.utils import log

_log = log.get("node.procs")


def gpu_pids(inv: Inventory, gpu: AmdGpu, drm_major: int = DRM_MAJOR) -> List[int]:
    try:
        return sorted({p.pid for p in inv.processes(gpu.index)})
    except NotImplementedError:
        return dev_users(drm_major, gpu.render_minor)


def dev_users(major: int, minor: int) -> List[int]:
    buf = (C.c_int32 * 4096)()
    n = C.c_int(0)
    rc = _native.host().gm_proc_dev_users(major, minor, buf, 4096, C.byref(n))
    if rc < 0:
        raise OSError(-rc, os.strerror(-rc))
    return sorted(int(buf[i]) for i in range(min(n.value, 4096)))


def filter_dev_users(pids: Sequence[int], major: int, minor: int) -> List[int]:
    """Of ``pids``, those with an open fd on char device ``major:minor``."""
    if not pids:
        return []
    arr = (C.c_int32 * len(pids))(*pids)
    out = (C.c_int32 * len(pids))()
    k = _native.host().gm_proc_filter_dev_users(arr, len(pids), major, minor, out)
    return [int(out[i]) for i in range(k)]


def busy_pids(inv: Inventory, gpus: Sequence[AmdGpu], container_pids: Iterable[int],
              drm_major: int = DRM_MAJOR) -> Dict[int, List[int]]:
    """GPU index → container PIDs that hold that GPU.

    Union of two sources: amdsmi's per-GPU process table (KFD contexts; may be filtered for an
    unprivileged caller) and an fd scan of *only the container's* PIDs for the GPU's render node
    (every HIP process keeps ``/dev/dri/renderD<N>`` open).
    """
    cpids = sorted(set(container_pids))
    out: Dict[int, List[int]] = {}
    for g in gpus:
        try:
            smi = set(p.pid for p in inv.processes(g.index))
        except NotImplementedError:
            smi = set()
        hit = set(cpids).intersection(smi)
        hit.update(filter_dev_users(cpids, drm_major, g.render_minor))
        if hit:
            out[g.index] = sorted(hit)
    return out


def signal_pids(pids: Sequence[int], sig: int) -> List[int]:
    if not pids:
        return []
    arr = (C.c_int32 * len(pids))(*pids)
    res = (C.c_int * len(pids))()
    _native.host().gm_proc_signal(arr, len(pids), sig, res)
    return [int(res[i]) for i in range(len(pids))]


def alive(pid: int) -> bool:
    return signal_pids([pid], 0)[0] == 0


async def terminate(pids: Sequence[int], sig: int = signal.SIGTERM, grace_s: float = 5.0) -> List[int]:
    """SIGTERM, wait up to ``grace_s``, then SIGKILL survivors. Returns PIDs signalled."""
    if not pids:
        return []
    signal_pids(pids, sig)
    deadline = asyncio.get_running_loop().time() + grace_s
    left = list(pids)
    while left and asyncio.get_running_loop().time() < deadline:
        await asyncio.sleep(0.02)
        left = [p for p in left if alive(p)]
    if left:
        _log.warning("SIGKILL after %.1fs grace: %s", grace_s, left)
        signal_pids(left, signal.SIGKILL)
    return list(pids)
