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
from typing import Dict, Iterable, List, Sequence, Tuple

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


def scan_devs(pids: Sequence[int], devs: Sequence[Tuple[int, int]]
              ) -> Tuple[List[List[bool]], List[int]]:
    """One read of each PID's fd table: (hits[pid][dev], PIDs whose table was unreadable)."""
    n, k = len(pids), len(devs)
    if not n or not k:
        return [[False] * k for _ in range(n)], []
    arr = (C.c_int32 * n)(*pids)
    mm = (C.c_uint32 * (2 * k))(*[v for d in devs for v in d])
    hits = (C.c_uint8 * (n * k))()
    bad = (C.c_int32 * n)()
    nbad = _native.host().gm_proc_scan_devs(arr, n, mm, k, hits, bad)
    if nbad < 0:
        raise OSError(-nbad, os.strerror(-nbad))
    return ([[bool(hits[i * k + j]) for j in range(k)] for i in range(n)],
            [int(bad[i]) for i in range(nbad)])


def busy_pids(inv: Inventory, gpus: Sequence[AmdGpu], container_pids: Iterable[int],
              drm_major: int = DRM_MAJOR, mode: str = "auto") -> Dict[int, List[int]]:
    """GPU index → container PIDs that hold that GPU.

    Primary source: one scan of *only the container's* PIDs for the GPUs' render nodes. A
    process cannot use a GPU without that fd (KFD binds a GPU's VM through its DRM render fd,
    and ROCr keeps it open for the process lifetime), so when every fd table is readable the
    scan is complete. amdsmi's per-GPU process table (KFD contexts, host PIDs) covers the PIDs
    whose fd table could not be read; ``mode="both"`` always takes the union (slower: amdsmi
    walks every KFD process on the node).
    """
    cpids = sorted(set(container_pids))
    hits, unreadable = scan_devs(cpids, [(drm_major, g.render_minor) for g in gpus])
    ask = set(cpids) if mode == "both" else set(unreadable)
    out: Dict[int, List[int]] = {}
    for j, g in enumerate(gpus):
        hit = {cpids[i] for i in range(len(cpids)) if hits[i][j]}
        if ask:
            try:
                hit.update(ask.intersection(p.pid for p in inv.processes(g.index)))
            except NotImplementedError:
                pass
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
