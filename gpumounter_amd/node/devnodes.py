"""Device-node injection into a running container's ``/dev``.

Reference: ``nsenter --target PID --mount sh -c "mknod -m 666 /dev/nvidiaN c 195 N"`` and
``… sh -c "rm /dev/nvidiaN"`` (reference: pkg/util/namespace/namespace.go:167-189), which needs
``mknod``/``sh`` inside the tenant image (FAQ.md:3-4) and forks three processes per GPU. Here one
C call handles every node of an attach: it resolves the container root through
``/proc/<pid>/root`` (or a setns helper thread, or — hermetic mode — a per-container directory),
walks ``dev/dri`` with ``O_NOFOLLOW`` (a hostile container cannot redirect the write with a
symlink), ``mknodat``s with an exact mode, and is idempotent.

Containers in their own user namespace (Kubernetes ``hostUsers: false``) cannot use such nodes:
their ``/dev`` is a tmpfs mounted inside that namespace, which the kernel treats as ``nodev``, so
an mknod'ed node there exists (and passes a naive read-back) but every ``open`` fails with EACCES.
The reference's ``mknod`` has the same defect. For those containers the writer switches to bind
mode (``GM_DEV_BIND``): the node is made once in a staging tmpfs the worker mounts itself, cloned
with ``open_tree`` and ``move_mount``ed over an empty placeholder in the container, owned by the
container's root as mapped through its ``uid_map``; the read-back then requires the mount.
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

    def __init__(self, mode: str = "procroot", host_dev: str = "", userns: str = "auto",
                 stage_dir: str = "", proc_root: str = "/proc") -> None:
        self.mode = mode
        self.userns = userns            # auto | bind | off (see _bind)
        self.stage_dir = stage_dir
        self.proc_root = proc_root
        self._staged = False
        self._own_userns = self._userns_id("self")
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
    def _array(nodes: Sequence[DeviceNode], owner: Tuple[int, int] = (-1, -1)):
        arr = (_native.DevNode * max(len(nodes), 1))()
        for i, n in enumerate(nodes):
            rel = n.path.lstrip("/").encode()
            if len(rel) >= 112:
                raise DevNodeError(f"path too long: {n.path}")
            arr[i].path = rel
            arr[i].major = n.major
            arr[i].minor = n.minor
            arr[i].mode = n.mode
            arr[i].uid, arr[i].gid = owner
        return arr

    # ------------------------------------------------------------------ which process
    def _mntns(self, pid) -> Optional[str]:
        try:
            return os.readlink(f"{self.proc_root}/{pid}/ns/mnt")
        except OSError:
            return None

    def root_pid(self, pids: Sequence[int]) -> int:
        """The process whose ``/proc/<pid>/root`` is the container's filesystem: the first of
        the cgroup's ``pids`` in a mount namespace other than this worker's. A process that was
        moved into the container's cgroup from outside it (a debugging tool, ``nsenter`` without
        ``-m``, a test probe) shares the worker's mount namespace, and its root is the worker's
        own: device nodes written through it would land in the worker's (or the host's) /dev.
        0 when there is no such process (the caller reports "no process to resolve its root
        from"). The reference always used the first PID of the cgroup (pkg/util/util.go:152)."""
        if self.mode == "emulate":
            return pids[0] if pids else 0
        own = self._mntns("self")
        for pid in pids:
            ns = self._mntns(pid)
            if ns is not None and ns != own:
                return pid
        return 0

    # ------------------------------------------------------------------ user-namespaced targets
    def _userns_id(self, pid) -> Optional[Tuple[int, int]]:
        try:
            st = os.stat(f"{self.proc_root}/{pid}/ns/user")
        except OSError:
            return None
        return st.st_dev, st.st_ino

    def _bind(self, t: Target) -> bool:
        """Bind mode for this target? ``bind``: always; ``off``: never; ``auto``: when the
        container's process lives in a user namespace other than the worker's."""
        if self.userns == "bind":
            return True
        if self.userns != "auto" or self.mode == "emulate" or t.root or t.pid <= 0:
            return False
        theirs = self._userns_id(t.pid)
        return theirs is not None and self._own_userns is not None and theirs != self._own_userns

    def _mapped_root(self, t: Target) -> Tuple[int, int]:
        """Host uid/gid of the container's root (its uid_map/gid_map entry for id 0), so the
        bind-mounted nodes show up as root-owned inside; (-1, -1) = leave as created."""
        if t.pid <= 0:
            return -1, -1
        out = []
        for f in ("uid_map", "gid_map"):
            host = -1
            try:
                with open(f"{self.proc_root}/{t.pid}/{f}") as fh:
                    for line in fh:
                        parts = line.split()
                        if len(parts) == 3 and int(parts[0]) == 0:
                            host = int(parts[1])
                            break
            except (OSError, ValueError):
                pass
            out.append(host)
        return out[0], out[1]

    def _ensure_stage(self) -> None:
        if self._staged:
            return
        if not self.stage_dir:
            raise DevNodeError("bind-mode device nodes need a staging directory "
                               "(devnode_stage_dir)")
        try:
            os.makedirs(os.path.dirname(self.stage_dir.rstrip("/")) or "/", exist_ok=True)
        except OSError as e:
            raise DevNodeError(f"staging directory {self.stage_dir}: {e.strerror}") from e
        rc = _native.host().gm_devnodes_stage(self.stage_dir.encode(), 1)
        if rc < 0:
            raise DevNodeError(f"staging tmpfs at {self.stage_dir}: {os.strerror(-rc)}")
        self._staged = True

    def _call(self, t: Target):
        """(flags, owner) for one target; sets up the staging tmpfs on first bind."""
        if not self._bind(t):
            return self.flags, (-1, -1)
        self._ensure_stage()
        return self.flags | _native.GM_DEV_BIND, self._mapped_root(t)

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
        flags, owner = self._call(t)
        res = (C.c_int * len(nodes))()
        fails = _native.host().gm_devnodes_create(pid, root, self._array(nodes, owner),
                                                  len(nodes), flags, res)
        results = [int(res[i]) for i in range(len(nodes))]
        if fails:
            bad = [(n.path, os.strerror(-r)) for n, r in zip(nodes, results) if r < 0]
            what = "bind mount" if flags & _native.GM_DEV_BIND else "mknod"
            raise DevNodeError(f"{what} failed: {bad}", results)
        return results

    def remove(self, t: Target, nodes: Sequence[DeviceNode]) -> List[int]:
        if not nodes:
            return []
        pid, root = self._target_args(t)
        flags, _ = self._call(t)
        res = (C.c_int * len(nodes))()
        fails = _native.host().gm_devnodes_remove(pid, root, self._array(nodes), len(nodes),
                                                  flags, res)
        results = [int(res[i]) for i in range(len(nodes))]
        if fails and not flags & _native.GM_DEV_BIND and \
                any(r == -errno.EBUSY for r in results) and self.mode != "emulate":
            # a bind-mounted node (attached while the container was handled in bind mode):
            # unmount those through the container's mount namespace
            busy = [i for i, r in enumerate(results) if r == -errno.EBUSY]
            self._ensure_stage()
            sub = [nodes[i] for i in busy]
            res2 = (C.c_int * len(sub))()
            _native.host().gm_devnodes_remove(pid, root, self._array(sub), len(sub),
                                              flags | _native.GM_DEV_BIND, res2)
            for k, i in enumerate(busy):
                results[i] = int(res2[k])
            fails = sum(1 for r in results if r < 0)
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
        rc = _native.host().gm_devnode_stat(pid, root, path.lstrip("/").encode(),
                                            self._call(t)[0],
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
        return [bool(s) for s in self.present_states(t, nodes)]

    def present_states(self, t: Target, nodes: Sequence[DeviceNode]) -> List[int]:
        """Per node: 0 absent, 1 present with the right major:minor, 2 in the host's guarded
        ``/dev`` (present, and never gpumounter's)."""
        if not nodes:
            return []
        pid, root = self._target_args(t)
        out = (C.c_uint8 * len(nodes))()
        rc = _native.host().gm_devnodes_present(pid, root, self._array(nodes), len(nodes),
                                                self._call(t)[0], out)
        if rc < 0:
            raise DevNodeError(f"read-back of {len(nodes)} nodes: {os.strerror(-rc)}")
        return [int(out[i]) for i in range(len(nodes))]
