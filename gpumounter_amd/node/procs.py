"""GPU busy detection and process termination.

Reference: busy ⇔ some NVML graphics/compute PID of the GPU is in the container's
``cgroup.procs`` (reference: pkg/util/util.go:152-196), with NVML re-initialised per query
(pkg/device/nvidia.go:58-87), and force-removal runs ``kill <pids>`` through nsenter
(namespace.go:191-201). Here the PID set comes from the cached amdsmi session
(``amdsmi_get_gpu_process_list``), with a ``/proc/*/fd`` scan for the GPU's render node as
fallback when amdsmi cannot report processes.

Both process tables, KFD's ``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>`` and amdsmi's list
(which reads the same table), name processes by their PID in the host's PID namespace. Measured
on an MI355X box (``profiles/r6_kfd_probe/``): a tenant that is PID 340 in its container is
``2370128`` in both tables, whose ``vram_<gpu_id>`` holds exactly its 256 MiB allocation. So the
tables are intersected with ``cgroup.procs`` only when the worker itself runs in the host PID
namespace (``hostPID: true``, :func:`host_pid_ns`); anywhere else a table PID could equal the
number of an unrelated container process. Force-removal pins the container's processes
with pidfds *before* the busy check (:class:`Pinned`): membership in the container's cgroup is
re-read after pinning, and SIGTERM, the liveness wait and the SIGKILL escalation all go through
those pidfds — so a PID the kernel recycles between the snapshot and the kill can never be hit.
Nothing in this module signals a bare PID number.
"""
from __future__ import annotations

import asyncio
import ctypes as C
import errno
import os
import select
import signal as _sig   # Pinned.signal shadows the module name inside the class body
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

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


KFD_PROC = "/sys/class/kfd/kfd/proc"
PROC_PID_INIT_INO = 0xEFFFFFFC      # the initial PID namespace's inode (linux/proc_ns.h)
_host_ns: Dict[str, bool] = {}
_warned: List[bool] = []          # the not-in-host-namespace warning, once per process


def host_pid_ns(proc_root: str = "/proc") -> bool:
    """This process runs in the host's (initial) PID namespace, so its PIDs are the numbers
    KFD and amdsmi report. ``/proc/self/status`` cannot tell (a container's /proc shows one
    NSpid too); the namespace inode can: the initial one has a fixed number."""
    if proc_root not in _host_ns:
        try:
            link = os.readlink(os.path.join(proc_root, "self/ns/pid"))
        except OSError:
            link = ""
        _host_ns[proc_root] = link == f"pid:[{PROC_PID_INIT_INO}]"
    return _host_ns[proc_root]


def kfd_table(root: str = KFD_PROC) -> Dict[int, Dict[int, int]]:
    """KFD's process table: KFD gpu_id → {host PID: VRAM bytes}. A process is listed under a
    GPU once it has bound that GPU (``vram_<gpu_id>`` in its directory). Raises OSError if the
    table cannot be read (no KFD, or sysfs not mounted at ``root``)."""
    out: Dict[int, Dict[int, int]] = {}
    for name in os.listdir(root):
        if not name.isdigit():
            continue
        pid = int(name)
        try:
            files = os.listdir(os.path.join(root, name))
        except OSError:
            continue                    # exited between the two reads
        for f in files:
            if not f.startswith("vram_") or not f[5:].isdigit():
                continue
            try:
                with open(os.path.join(root, name, f), "rb") as fh:
                    vram = int(fh.read().strip() or 0)
            except (OSError, ValueError):
                continue
            out.setdefault(int(f[5:]), {})[pid] = vram
    return out


def busy_pids(inv: Inventory, gpus: Sequence[AmdGpu], container_pids: Iterable[int],
              drm_major: int = DRM_MAJOR, mode: str = "auto", kfd_root: str = "",
              tables: bool = True) -> Dict[int, List[int]]:
    """GPU index → container PIDs that hold that GPU.

    Primary source: one scan of *only the container's* PIDs for the GPUs' render nodes. A
    process cannot use a GPU without that fd (KFD binds a GPU's VM through its DRM render fd,
    and ROCr keeps it open for the process lifetime), so when every fd table is readable the
    scan is complete. The process tables cover the PIDs whose fd table could not be read:
    KFD's sysfs table when ``kfd_root`` is given and readable (a few small reads), else
    amdsmi's. The worker passes ``kfd_root`` only with the real amdsmi library: the mock
    library's GPUs are not this node's KFD nodes.
    ``mode="both"`` always takes the union. ``tables=False`` (the worker is not in the host
    PID namespace, see the module docstring) leaves the tables out: their PIDs are not this
    namespace's.
    """
    cpids = sorted(set(container_pids))
    hits, unreadable = scan_devs(cpids, [(drm_major, g.render_minor) for g in gpus])
    ask = set(cpids) if mode == "both" else set(unreadable)
    if ask and not tables:
        if not _warned:
            _warned.append(True)
            _log.warning("busy check: not in the host PID namespace, so the KFD/amdsmi process "
                         "tables cannot vouch for PIDs such as %s (run the worker with "
                         "hostPID: true)", sorted(ask)[:8])
        ask = set()
    kfd: Optional[Dict[int, Dict[int, int]]] = None
    if ask and kfd_root:
        try:
            kfd = kfd_table(kfd_root)
        except OSError:
            kfd = None
    out: Dict[int, List[int]] = {}
    for j, g in enumerate(gpus):
        hit = {cpids[i] for i in range(len(cpids)) if hits[i][j]}
        if ask:
            if kfd is not None and g.kfd_gpu_id:
                hit.update(ask.intersection(kfd.get(g.kfd_gpu_id, {})))
            else:
                try:
                    hit.update(ask.intersection(p.pid for p in inv.processes(g.index)))
                except NotImplementedError:
                    pass
        if hit:
            out[g.index] = sorted(hit)
    return out


def start_time(pid: int) -> int:
    """Start time of ``pid`` in clock ticks since boot (``/proc/<pid>/stat`` field 22), or 0 if
    there is no such process. (PID, start time) names one process for the node's uptime: a
    recycled PID has a later start time. Used where no pidfd can be held — across a worker
    restart, for the PIDs a drained placeholder waits on."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as fh:
            raw = fh.read()
    except OSError:
        return 0
    # comm may contain spaces and parentheses: the fields after it start at the last ')'
    rest = raw[raw.rfind(b")") + 2:].split()
    try:
        return int(rest[19])
    except (IndexError, ValueError):
        return 0


def same_process(pid: int, started: int) -> bool:
    """``pid`` is still the process that had start time ``started`` (and has not exited)."""
    st = start_time(pid)
    if not st or st != started:
        return False
    try:
        with open(f"/proc/{pid}/stat", "rb") as fh:
            raw = fh.read()
        return raw[raw.rfind(b")") + 2:][:1] != b"Z"      # a zombie holds no fds any more
    except OSError:
        return False


class Pinned:
    """pidfds for a snapshot of PIDs, held from the busy check through the kill.

    A pidfd refers to one process, not to a number: once that process has exited, signalling
    through it fails with ESRCH even if the PID was handed to someone else. So the only window
    left is between reading ``cgroup.procs`` and ``pidfd_open``; :meth:`restrict` closes it by
    re-reading the cgroup *after* pinning (a pinned, unreaped process keeps its PID, so a PID
    still listed is the pinned process)."""

    def __init__(self, pids: Iterable[int]) -> None:
        self.fds: Dict[int, int] = {}
        for p in sorted(set(pids)):
            try:
                self.fds[p] = os.pidfd_open(p)
            except ProcessLookupError:
                continue            # already gone: nothing to pin, nothing to kill
            except OSError as e:
                if e.errno != errno.ESRCH:
                    raise

    def pids(self) -> List[int]:
        return sorted(self.fds)

    def restrict(self, still: Iterable[int]) -> List[int]:
        """Keep only PIDs still listed (re-read after pinning); returns those dropped."""
        keep = set(still)
        dropped = [p for p in self.fds if p not in keep]
        for p in dropped:
            os.close(self.fds.pop(p))
        return dropped

    def exited(self, pid: int) -> bool:
        fd = self.fds.get(pid)
        if fd is None:
            return True
        # a pidfd polls readable once its process exits; poll(2), not select(2): the drain
        # keeper holds pidfds for long, and select() refuses any fd ≥ FD_SETSIZE (1024)
        p = select.poll()
        p.register(fd, select.POLLIN)
        return bool(p.poll(0))

    def signal(self, pids: Sequence[int], sig: int) -> List[int]:
        """0 or -errno per PID; never reaches a process other than the pinned one."""
        out = []
        for p in pids:
            fd = self.fds.get(p)
            if fd is None:
                out.append(-errno.ESRCH)
                continue
            try:
                _sig.pidfd_send_signal(fd, sig)
                out.append(0)
            except OSError as e:
                out.append(-(e.errno or errno.ESRCH))
        return out

    async def wait_exit(self, pids: Sequence[int], timeout: float) -> List[int]:
        """Wait up to ``timeout`` s for the pinned processes to exit (their pidfds become
        readable: no polling); returns the ones still running."""
        live = [p for p in pids if p in self.fds and not self.exited(p)]
        if not live or timeout <= 0:
            return live
        loop = asyncio.get_running_loop()
        done = loop.create_future()
        left = set(live)

        def on_exit(pid: int) -> None:
            loop.remove_reader(self.fds[pid])
            left.discard(pid)
            if not left and not done.done():
                done.set_result(None)
        for p in live:
            loop.add_reader(self.fds[p], on_exit, p)
        try:
            await asyncio.wait_for(asyncio.shield(done), timeout)
        except asyncio.TimeoutError:
            pass
        finally:
            for p in list(left):
                loop.remove_reader(self.fds[p])
        return sorted(p for p in live if not self.exited(p))

    async def reap(self, pids: Sequence[int], sig: int = _sig.SIGTERM, grace_s: float = 5.0,
                   kill_wait_s: float = 2.0, already_signalled: bool = False,
                   sigkill: bool = True) -> Tuple[List[int], List[int]]:
        """``sig``; wait up to ``grace_s`` for the pinned processes to exit; SIGKILL the rest
        and wait up to ``kill_wait_s`` for them to go. Returns (PIDs that needed SIGKILL, PIDs
        still running after it — uninterruptible sleep). The pidfds stay open: a caller that
        must wait on survivors keeps them, then calls :meth:`close`. ``sigkill=False`` withholds
        the SIGKILL (fault injection: a process the kernel cannot kill yet)."""
        live = [p for p in pids if p in self.fds]
        if not already_signalled:
            self.signal(live, sig)
        live = await self.wait_exit(live, grace_s)
        if not live:
            return [], []
        _log.warning("SIGKILL after %.1fs grace: %s", grace_s, live)
        if sigkill:
            self.signal(live, _sig.SIGKILL)
        survivors = await self.wait_exit(live, kill_wait_s)
        if survivors:
            _log.error("still running %.1fs after SIGKILL (uninterruptible?): %s",
                       kill_wait_s, survivors)
        return live, survivors

    def keep_only(self, pids: Iterable[int]) -> None:
        """Close every pidfd except those of ``pids`` (the ones a drain still waits on)."""
        want = set(pids)
        for p in [p for p in self.fds if p not in want]:
            os.close(self.fds.pop(p))

    def close(self) -> None:
        for fd in self.fds.values():
            try:
                os.close(fd)
            except OSError:
                pass
        self.fds.clear()

    def __del__(self) -> None:
        self.close()
