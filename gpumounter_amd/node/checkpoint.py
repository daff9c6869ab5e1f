"""The kubelet device manager's checkpoint: the node's GPU ledger without a kubelet RPC.

The reference learns which GPUs a slave pod got by dialing the kubelet's PodResources socket and
listing every pod on the node, once per slave pod and again per query (reference:
pkg/util/gpu/collector/collector.go:90-138, allocator.go:86-94). Kubelets rate-limit that server
(100 qps, burst 10, RESOURCE_EXHAUSTED beyond), so a ledger read per attach caps a node at a
few dozen attaches per second and competes with every other node agent for the same budget.

The device manager persists the very same allocation state it serves over PodResources: after
every device-plugin ``Allocate`` at admission it rewrites
``/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint`` (written to a temporary file and
renamed into place, so a reader never sees a torn file) with one entry per (pod UID, container,
resource)::

    {"Data": {"PodDeviceEntries": [{"PodUID": "...", "ContainerName": "...",
                                    "ResourceName": "amd.com/gpu",
                                    "DeviceIDs": {"0": ["0000:05:00.0"]},   # NUMA → IDs
                                    "AllocResp": "<base64>"}],
              "RegisteredDevices": {"amd.com/gpu": [...]}},
     "Checksum": 123}

(``DeviceIDs`` was a flat list before Kubernetes 1.20; both are read). The worker already
mounts that directory for the device-plugin socket. Placeholders are looked up by pod UID, so
a stale entry of a deleted pod can never match a fresh placeholder, and an inotify watch on the
directory wakes admission waiters the moment the kubelet renames a new checkpoint in.

PodResources stays the authority. The checkpoint serves admission and non-authoritative ledger
views (``/audit``, leases). PodResources serves the reconciler, rollbacks and worker start-up,
and every one of those reads is compared with the checkpoint pod by pod. The checkpoint is no
longer trusted after three reads in a row disagree, or after three placeholders in a row that
the apiserver shows as admitted have no entry in it. PodResources is also read whenever the
file is missing or unreadable.
"""
from __future__ import annotations

import asyncio
import ctypes as C
import ctypes.util
import json
import os
import struct
import time
from typing import Callable, Dict, List, Optional, Tuple

from gpumounter_amd.utils import calls, log

_log = log.get("node.checkpoint")

CHECKPOINT_NAME = "kubelet_internal_checkpoint"

# <sys/inotify.h>
IN_CLOSE_WRITE = 0x00000008
IN_MOVED_TO = 0x00000080
IN_CREATE = 0x00000100
IN_Q_OVERFLOW = 0x00004000
IN_NONBLOCK = 0o4000
IN_CLOEXEC = 0o2000000
_EVENT = struct.Struct("iIII")        # wd, mask, cookie, len


class CheckpointFormatError(ValueError):
    pass


def parse(blob: bytes, resource: str) -> Dict[str, Tuple[str, ...]]:
    """pod UID → device IDs of ``resource`` (every container of the pod, entry order)."""
    try:
        doc = json.loads(blob)
        entries = doc["Data"].get("PodDeviceEntries") or []
    except (ValueError, KeyError, TypeError, AttributeError) as e:
        raise CheckpointFormatError(f"not a device-manager checkpoint: {e}") from e
    out: Dict[str, list] = {}
    for e in entries:
        if not isinstance(e, dict):
            raise CheckpointFormatError("PodDeviceEntries holds a non-object")
        if e.get("ResourceName") != resource:
            continue
        ids = e.get("DeviceIDs")
        if isinstance(ids, dict):               # ≥ 1.20: NUMA node → IDs
            flat = [i for k in sorted(ids, key=lambda k: (len(k), k)) for i in (ids[k] or [])]
        elif isinstance(ids, list):             # < 1.20: flat list
            flat = list(ids)
        elif ids is None:
            flat = []
        else:
            raise CheckpointFormatError(f"DeviceIDs of type {type(ids).__name__}")
        uid = e.get("PodUID")
        if not isinstance(uid, str) or not all(isinstance(i, str) for i in flat):
            raise CheckpointFormatError("PodUID/DeviceIDs are not strings")
        out.setdefault(uid, []).extend(flat)
    return {k: tuple(v) for k, v in out.items()}


def render(entries, registered: Optional[Dict[str, list]] = None) -> bytes:
    """The kubelet's on-disk form of ``entries`` = [(uid, container, resource, {numa: ids})]
    (the fake kubelet writes it; ``Checksum`` is not the kubelet's hash and is never checked)."""
    data = {"PodDeviceEntries": [{"PodUID": uid, "ContainerName": c, "ResourceName": r,
                                  "DeviceIDs": {str(k): list(v) for k, v in per_numa.items()},
                                  "AllocResp": ""}
                                 for uid, c, r, per_numa in entries],
            "RegisteredDevices": registered or {}}
    body = json.dumps(data, sort_keys=True)
    return json.dumps({"Data": data, "Checksum": sum(body.encode()) & 0x7fffffff}).encode()


def write_atomic(path: str, blob: bytes) -> None:
    """tmp + rename in the checkpoint's directory, as the kubelet's file store does."""
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as fh:
        fh.write(blob)
    os.replace(tmp, path)


class DeviceCheckpoint:
    """Reader of the device-manager checkpoint with an inotify wake-up.

    :meth:`lookup` reads the file on every call and parses it again only when its bytes
    changed, so a read costs one small ``read`` in the steady state."""

    CHECKPOINT_MISSES = 3

    def __init__(self, path: str, resource: str) -> None:
        self.path = path
        self.resource = resource
        self._blob: Optional[bytes] = None
        self._by_uid: Dict[str, Tuple[str, ...]] = {}
        self.parses = 0
        self.errors = 0
        self.trusted = True          # cleared when the kubelet is seen not to maintain it
        self.mismatches = 0
        self._fd = -1
        self._loop = None

    # ------------------------------------------------------------------------ reads
    def snapshot(self) -> Optional[Dict[str, Tuple[str, ...]]]:
        """uid → IDs, or None if the file is absent or unreadable.

        The file is read on every call and parsed again only when its bytes changed. Stat
        metadata cannot stand in for the content: the kubelet's tmp-and-rename reuses the inode
        number just freed, two rewrites within one timestamp tick share an mtime, and a rewrite
        that swaps one UID for another keeps the size."""
        t = time.monotonic()
        calls.record("checkpoint read", t, t)
        try:
            with open(self.path, "rb") as fh:
                blob = fh.read()
        except OSError:
            self._blob = None
            return None
        if blob != self._blob:
            try:
                self._by_uid = parse(blob, self.resource)
            except CheckpointFormatError as e:
                self.errors += 1
                if self.errors == 1 or self.errors % 100 == 0:
                    _log.warning("device-manager checkpoint %s unreadable: %s", self.path, e)
                self._blob = None
                return None
            self._blob = blob
            self.parses += 1
        return self._by_uid

    def lookup(self, uid: str) -> Optional[Tuple[str, ...]]:
        """The pod's device IDs; None when unknown (not admitted yet, or no usable file)."""
        if not self.trusted:
            return None
        snap = self.snapshot()
        if snap is None:
            return None
        return snap.get(uid) or None

    def by_name(self, pods) -> Optional[Dict[Tuple[str, str], List[str]]]:
        """The ledger keyed like a PodResources List — (namespace, name) → IDs — for the given
        pod objects (the informers' caches); None when the checkpoint cannot be used."""
        if not self.trusted:
            return None
        snap = self.snapshot()
        if snap is None:
            return None
        out: Dict[Tuple[str, str], List[str]] = {}
        for p in pods:
            md = p["metadata"]
            ids = snap.get(md.get("uid", ""))
            if ids:
                out[(md["namespace"], md["name"])] = list(ids)
        return out

    def cross_check(self, listed: Dict[Tuple[str, str], List[str]],
                    uid_of: Callable[[Tuple[str, str]], Optional[str]]) -> bool:
        """Compare an authoritative PodResources view with the checkpoint, pod by pod (for the
        pods whose UID is known). ``CHECKPOINT_MISSES`` disagreeing reads in a row distrust
        it — a single one can be the microseconds between the kubelet's in-memory update and
        its rename. Returns whether this read agreed."""
        if not self.trusted:
            return False
        snap = self.snapshot()
        bad = snap is None and bool(listed)
        for key, ids in listed.items():
            if bad:
                break
            uid = uid_of(key)
            if uid and sorted(snap.get(uid, ())) != sorted(ids):
                bad = True
        if not bad:
            self.mismatches = 0
            return True
        self.mismatches += 1
        if self.mismatches >= self.CHECKPOINT_MISSES:
            self.distrust(f"{self.mismatches} PodResources reads in a row disagreed with it")
        return False

    def distrust(self, why: str) -> None:
        if self.trusted:
            _log.warning("not using the device-manager checkpoint %s any more: %s", self.path, why)
        self.trusted = False

    # ------------------------------------------------------------------------ inotify
    def watch(self, on_change: Callable[[], None]) -> bool:
        """Call ``on_change`` (on the running loop) whenever the kubelet renames a new checkpoint
        in. False when the directory cannot be watched; lookups still work, waiters then rely on
        pod events and their backoff."""
        d = os.path.dirname(self.path) or "."
        if not os.path.isdir(d):
            return False
        libc = C.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        fd = libc.inotify_init1(IN_NONBLOCK | IN_CLOEXEC)
        if fd < 0:
            _log.info("inotify unavailable: %s", os.strerror(C.get_errno()))
            return False
        if libc.inotify_add_watch(fd, d.encode(), IN_MOVED_TO | IN_CLOSE_WRITE | IN_CREATE) < 0:
            _log.info("inotify watch on %s: %s", d, os.strerror(C.get_errno()))
            os.close(fd)
            return False
        name = os.path.basename(self.path).encode()
        self._fd = fd
        self._loop = asyncio.get_running_loop()

        def readable() -> None:
            hit = False
            while True:
                try:
                    buf = os.read(fd, 4096)
                except BlockingIOError:
                    break
                except OSError:
                    return
                if not buf:
                    break
                off = 0
                while off + _EVENT.size <= len(buf):
                    _, mask, _, ln = _EVENT.unpack_from(buf, off)
                    nm = buf[off + _EVENT.size:off + _EVENT.size + ln].rstrip(b"\0")
                    off += _EVENT.size + ln
                    if nm == name or mask & IN_Q_OVERFLOW:
                        hit = True
            if hit:
                on_change()

        self._loop.add_reader(fd, readable)
        return True

    def close(self) -> None:
        if self._fd >= 0:
            if self._loop is not None and not self._loop.is_closed():
                self._loop.remove_reader(self._fd)
            os.close(self._fd)
            self._fd = -1
