"""Keep hot-mounted devices in the container unit's systemd DeviceAllow= list.

With the systemd cgroup driver the container's cgroup is a transient scope
(``cri-containerd-<id>.scope`` …) and systemd owns its device policy. Whenever systemd re-realises
the unit (``daemon-reload``, any property change) it rewrites v1 ``devices.allow/deny`` or attaches
a new v2 device program from DeviceAllow=, and a grant made behind its back is lost.
The reference only supports cgroupfs + cgroup v1 and never met this (reference:
pkg/util/cgroup/cgroup.go:78-118).

:class:`SystemdPersistingBackend` wraps the real rule backend: the kernel-side grant stays on the
request path (it is what makes the device usable now), and the unit's DeviceAllow= is brought in
line afterwards on a background thread (``SetUnitProperties``, runtime) through the native D-Bus
client in ``native/src/gm_sdbus.cpp``. Updates for one unit coalesce; only paths gpumounter itself
manages are ever added or removed, so the runtime's own entries are left alone.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

from gpumounter_amd import _native
from gpumounter_amd.node.cgroup import DeviceRuleBackend
from gpumounter_amd.utils import log

_log = log.get("node.systemd")

DEFAULT_BUSES = ("/run/systemd/private", "/run/dbus/system_bus_socket")
UNIT_SUFFIXES = (".scope", ".service")


class SystemdError(RuntimeError):
    pass


def unit_of(cgdir: str) -> Optional[str]:
    """The systemd unit owning a container cgroup directory (None for cgroupfs-driver paths)."""
    name = os.path.basename(cgdir.rstrip("/"))
    return name if name.endswith(UNIT_SUFFIXES) else None


def find_bus(explicit: str = "") -> Optional[str]:
    if explicit:
        return explicit
    for p in DEFAULT_BUSES:
        if os.path.exists(p):
            return p
    return None


class SystemdBus:
    """The two calls used here, over systemd's private socket or the system bus."""

    def __init__(self, path: str) -> None:
        self.path = path

    def device_allow(self, unit: str) -> List[Tuple[str, str]]:
        lib = _native.host()
        err = C.create_string_buffer(512)
        cap = 1 << 16
        while True:
            out = C.create_string_buffer(cap)
            rc = lib.gm_sd_get_device_allow(self.path.encode(), unit.encode(), out, cap, err, 512)
            if rc == -28 and cap < (1 << 22):   # ENOSPC
                cap *= 4
                continue
            break
        if rc < 0:
            raise SystemdError(f"DeviceAllow of {unit}: {err.value.decode() or os.strerror(-rc)}")
        entries = []
        for line in out.value.decode().splitlines():
            path, _, perm = line.partition("\t")
            entries.append((path, perm))
        return entries

    def set_device_allow(self, unit: str, entries: Sequence[Tuple[str, str]], reset: bool) -> None:
        lib = _native.host()
        paths = (C.c_char_p * max(len(entries), 1))(*[p.encode() for p, _ in entries])
        perms = (C.c_char_p * max(len(entries), 1))(*[m.encode() for _, m in entries])
        err = C.create_string_buffer(512)
        rc = lib.gm_sd_set_device_allow(self.path.encode(), unit.encode(), paths, perms,
                                        len(entries), 1 if reset else 0, err, 512)
        if rc < 0:
            raise SystemdError(f"SetUnitProperties({unit}): "
                               f"{err.value.decode() or os.strerror(-rc)}")


class DeviceAllowSync:
    """Background, coalescing DeviceAllow= updater (one thread; latest desired state per unit)."""

    def __init__(self, bus: SystemdBus, retry_s: float = 2.0, max_attempts: int = 5) -> None:
        self.bus = bus
        self.retry_s = retry_s
        self.max_attempts = max_attempts
        self._pending: Dict[str, Tuple[Set[str], Set[str], int]] = {}  # unit → (want, retired, tries)
        self._cv = threading.Condition()
        self._busy = 0
        self._stop = False
        self.synced = 0
        self.errors = 0
        self.last_error = ""
        self._thread = threading.Thread(target=self._run, name="gm-systemd-sync", daemon=True)
        self._thread.start()

    def update(self, unit: str, want: Iterable[str], revoked: Iterable[str]) -> None:
        want = set(want)
        with self._cv:
            _, retired, _ = self._pending.get(unit, (set(), set(), 0))
            retired = (retired | set(revoked)) - want
            self._pending[unit] = (want, retired, 0)
            self._cv.notify_all()

    def flush(self, timeout: float = 10.0) -> bool:
        """Wait until every queued unit was synced (or gave up). True if nothing is left."""
        end = time.monotonic() + timeout
        with self._cv:
            while self._pending or self._busy:
                left = end - time.monotonic()
                if left <= 0:
                    return False
                self._cv.wait(left)
        return True

    def stop(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(timeout=5)

    def sync_unit(self, unit: str, want: Set[str], retired: Set[str]) -> bool:
        """One reconciliation of the unit's list. Returns True if systemd was changed."""
        cur = self.bus.device_allow(unit)
        keep = [(p, m) for p, m in cur if p not in retired or p in want]
        have = {p for p, _ in keep}
        add = [(p, "rw") for p in sorted(want) if p not in have]
        if len(keep) != len(cur):
            self.bus.set_device_allow(unit, keep + add, reset=True)
            return True
        if add:
            self.bus.set_device_allow(unit, add, reset=False)
            return True
        return False

    def _run(self) -> None:
        while True:
            with self._cv:
                while not self._pending and not self._stop:
                    self._cv.wait()
                if self._stop:
                    return
                unit, (want, retired, tries) = next(iter(self._pending.items()))
                del self._pending[unit]
                self._busy += 1
            try:
                changed = self.sync_unit(unit, want, retired)
                self.synced += 1
                log.kv(_log, 10, "systemd DeviceAllow synced", unit=unit, changed=changed,
                       devices=len(want))
            except Exception as e:  # noqa: BLE001
                self.errors += 1
                self.last_error = str(e)
                _log.warning("systemd DeviceAllow of %s not updated (try %d): %s", unit,
                             tries + 1, e)
                if tries + 1 < self.max_attempts:
                    time.sleep(self.retry_s)
                    with self._cv:
                        if unit not in self._pending:   # a newer update supersedes the retry
                            self._pending[unit] = (want, retired, tries + 1)
            finally:
                with self._cv:
                    self._busy -= 1
                    self._cv.notify_all()


class SystemdPersistingBackend(DeviceRuleBackend):
    """Kernel grant through ``inner`` now; the unit's DeviceAllow= follows in the background."""

    def __init__(self, inner: DeviceRuleBackend, sync: DeviceAllowSync) -> None:
        self.inner = inner
        self.sync = sync
        self.name = f"{inner.name}+systemd"

    def apply(self, cgdir, grant, revoke, desired):
        self.inner.apply(cgdir, grant, revoke, desired)
        unit = unit_of(cgdir)
        if unit is not None:
            self.sync.update(unit, [n.path for n in desired], [n.path for n in revoke])

    def allowed(self, cgdir):
        return self.inner.allowed(cgdir)

    def fingerprint(self, cgdir):
        return self.inner.fingerprint(cgdir)

    def installed(self, cgdir):
        return self.inner.installed(cgdir)

    def prune(self):
        return self.inner.prune()

    def sweep_pins(self, cgroup_root: str):
        sweep = getattr(self.inner, "sweep_pins", None)
        return sweep(cgroup_root) if sweep is not None else []


def maybe_wrap(backend: DeviceRuleBackend, mode: str, bus_path: str,
               driver: str) -> DeviceRuleBackend:
    """Apply the ``systemd_device_allow`` policy: off | on | auto (a bus socket exists and the
    cgroup driver may be systemd)."""
    if mode == "off" or (mode == "auto" and driver == "cgroupfs"):
        return backend
    bus = find_bus(bus_path)
    if bus is None:
        if mode == "on":
            raise SystemdError("systemd_device_allow=on but no systemd bus socket found "
                               f"(tried {bus_path or ', '.join(DEFAULT_BUSES)})")
        return backend
    _log.info("systemd DeviceAllow persistence on via %s", bus)
    return SystemdPersistingBackend(backend, DeviceAllowSync(SystemdBus(bus)))
