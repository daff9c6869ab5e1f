"""Device-node injection into a running container's ``/dev``.

Reference: ``nsenter --target PID --mount sh -c "mknod -m 666 /dev/nvidiaN c 195 N"`` and
``… sh -c "rm /dev/nvidiaN"`` (reference: pkg/util/namespace/namespace.go:167-189), which needs
``mknod``/``sh`` inside the tenant image (FAQ.md:3-4) and forks three processes per GPU. Here one
C call handles every node of an attach: it resolves the container root through
``/proc/<pid>/root`` (or a setns helper thread, or — hermetic mode — a per-container directory),
walks ``dev/dri`` with ``O_NOFOLLOW`` (a hostile container cannot redirect the write with a
symlink), ``mknodat``s with an exact mode, and is idempotent.
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

from gpumounter_amd import _native
from gpumounter_amd.models.device import DeviceNode
from gpumounter_amd.utils import log


class DevNodeError(RuntimeError):
    def __init__(self, msg: str, results: Sequence[int] = ()):
        super().__init__(msg)
        self.results = list(results)


@dataclass(frozen=True)
class Target:
    """Where a container's filesystem is reachable from the worker."""

    pid: int = 0               # a process inside the container (procroot / setns modes)
    root: str = ""             # explicit root directory (hermetic / test mode)


CREATED, PRESENT, SHARED_HOST = 0, 1, 2

_log = log.get("node.devnodes")


class DevNodeWriter:
    """``host_dev``: the host's ``/dev`` as the worker sees it. A container directory that *is*
    that ``/dev`` (or its ``dri/``) — a hostPath ``/dev`` bind, a privileged runtime's — is never
    written: creates and unlinks there report :data:`SHARED_HOST` and leave the host's nodes be.
    The guard is process-wide in the native layer (the last writer constructed sets or clears
    it; a worker process has exactly one)."""

    def __init__(self, mode: str = "procroot", host_dev: str = "") -> None:
        self.mode = mode
        self.flags = 0
        if mode == "setns":
            self.flags |= _native.GM_DEV_VIA_SETNS
        if mode == "emulate":
            self.flags |= _native.GM_DEV_EMULATE
        self.host_dev = host_dev
        # always (re)set: a writer without host_dev clears a guard an earlier one left, whose
        # directory may be gone and its inode number reused by an unrelated directory
        rc = _native.host().gm_devnodes_guard(host_dev.encode() if host_dev else None)
        if rc < 0:
            _log.warning("host /dev guard off: cannot read %s (%s)", host_dev, os.strerror(-rc))
        self.guarded = max(rc, 0)

    @staticmethod
    def _array(nodes: Sequence[DeviceNode]):
        arr = (_native.DevNode * max(len(nodes), 1))()
        for i, n in enumerate(nodes):
            rel = n.path.lstrip("/").encode()
            if len(rel) >= 112:
                raise DevNodeError(f"path too long: {n.path}")
            arr[i].path = rel
            arr[i].major = n.major
            arr[i].minor = n.minor
            arr[i].mode = n.mode
            arr[i].uid = -1
            arr[i].gid = -1
        return arr

    def _target_args(self, t: Target) -> Tuple[int, Optional[bytes]]:
        if t.root:
            return 0, t.root.encode()
        if t.pid <= 0:
            raise DevNodeError("container has no process to resolve its root from "
                               "(empty cgroup.procs)")
        return t.pid, None

    def create(self, t: Target, nodes: Sequence[DeviceNode]) -> List[int]:
        if not nodes:
            return []
        pid, root = self._target_args(t)
        res = (C.c_int * len(nodes))()
        fails = _native.host().gm_devnodes_create(pid, root, self._array(nodes), len(nodes),
                                                  self.flags, res)
        results = [int(res[i]) for i in range(len(nodes))]
        if fails:
            bad = [(n.path, os.strerror(-r)) for n, r in zip(nodes, results) if r < 0]
            raise DevNodeError(f"mknod failed: {bad}", results)
        return results

    def remove(self, t: Target, nodes: Sequence[DeviceNode]) -> List[int]:
        if not nodes:
            return []
        pid, root = self._target_args(t)
        res = (C.c_int * len(nodes))()
        fails = _native.host().gm_devnodes_remove(pid, root, self._array(nodes), len(nodes),
                                                  self.flags, res)
        results = [int(res[i]) for i in range(len(nodes))]
        if fails:
            # ESRCH/ENOENT on the root means the container is gone: nothing left to remove
            if all(r in (-errno.ESRCH, -errno.ENOENT) for r in results if r < 0):
                return [PRESENT if r < 0 else r for r in results]
            bad = [(n.path, os.strerror(-r)) for n, r in zip(nodes, results) if r < 0]
            raise DevNodeError(f"unlink failed: {bad}", results)
        shared = [n.path for n, r in zip(nodes, results) if r == SHARED_HOST]
        if shared:
            _log.warning("not unlinking %s: the container's directory is the host's /dev", shared)
        return results

    def stat(self, t: Target, path: str) -> Tuple[int, int, int, int]:
        """(kind, major, minor, mode): kind 0 absent, 1 char device, 2 marker, 3 other."""
        pid, root = self._target_args(t)
        kind, ma, mi, mode = C.c_int(0), C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
        rc = _native.host().gm_devnode_stat(pid, root, path.lstrip("/").encode(), self.flags,
                                            C.byref(kind), C.byref(ma), C.byref(mi),
                                            C.byref(mode))
        if rc < 0:
            raise DevNodeError(f"stat {path}: {os.strerror(-rc)}")
        return kind.value, ma.value, mi.value, mode.value

    def present(self, t: Target, node: DeviceNode) -> bool:
        kind, ma, mi, _ = self.stat(t, node.path)
        return kind in (1, 2) and ma == node.major and mi == node.minor

    def present_many(self, t: Target, nodes: Sequence[DeviceNode]) -> List[bool]:
        """:meth:`present` for a whole node set in one native call (one root resolution). A
        node in a directory that is the host's own ``/dev`` counts as present: create leaves
        it to the host (:data:`SHARED_HOST`) and so does the read-back."""
        if not nodes:
            return []
        pid, root = self._target_args(t)
        out = (C.c_uint8 * len(nodes))()
        rc = _native.host().gm_devnodes_present(pid, root, self._array(nodes), len(nodes),
                                                self.flags, out)
        if rc < 0:
            raise DevNodeError(f"read-back of {len(nodes)} nodes: {os.strerror(-rc)}")
        return [bool(out[i]) for i in range(len(nodes))]
