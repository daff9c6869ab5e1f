"""Container cgroup resolution and device-access backends (cgroup v1 and v2).

Reference: the cgroup path is *computed* from the pod QoS and an env-selected driver, assuming
``docker-<id>.scope`` for systemd and the v1 ``/sys/fs/cgroup/devices`` mount only; rules are
written by forking ``sh -c "echo 'c 195:N rw' > …/devices.allow"`` (reference:
pkg/util/cgroup/cgroup.go:78-169). Here:

* :class:`CgroupResolver` auto-detects v1/v2 and the driver, tries the computed QoS path for every
  runtime naming scheme (``docker-``, ``cri-containerd-``, ``crio-`` scopes; cgroupfs ids) and
  falls back to a directory search under the pod cgroup — runtime-agnostic;
* :class:`V1Backend` writes rules in-process (one ``write(2)`` per rule, C++);
* :class:`V2BpfBackend` swaps in a generated ``BPF_PROG_TYPE_CGROUP_DEVICE`` allow-list that
  tail-calls the runtime's original program (C++, raw ``bpf(2)``);
* :class:`V2RecordingBackend` produces the identical program bytes without loading them (for
  unprivileged hosts and hermetic tests), storing the rule set next to the fake cgroup.
"""
from __future__ import annotations

import ctypes as C
import errno
import functools
import glob
import json
import os
from abc import ABC, abstractmethod
from typing import Dict, FrozenSet, Iterable, List, Optional, Sequence, Set, Tuple

from gpumounter_amd import _native
from gpumounter_amd.models.device import DeviceNode
from gpumounter_amd.models.pod import (QOS_BESTEFFORT, QOS_BURSTABLE, ContainerRef, qos_class,
                                       uid_of)
from gpumounter_amd.node import bpfvm
from gpumounter_amd.utils import log, trace

_log = log.get("node.cgroup")

RUNTIME_SCOPE_PREFIXES = ("cri-containerd-", "docker-", "crio-", "containerd-", "")
FAKE_MARKER = ".gm_fake"
BPF_STATE = "gm.bpf.json"


class CgroupError(RuntimeError):
    pass


def _esc(s: str) -> str:
    return s.replace("-", "_")


class CgroupResolver:
    def __init__(self, root: str = "/sys/fs/cgroup", mode: str = "auto", driver: str = "auto",
                 proc_root: str = "/proc"):
        self.root = root
        self.proc_root = proc_root
        self.mode = self.detect_mode(root) if mode == "auto" else mode
        self.base = os.path.join(root, "devices") if self.mode == "v1" else root
        self.driver = driver
        self._cache: Dict[Tuple[str, str], str] = {}

    @staticmethod
    def detect_mode(root: str) -> str:
        if os.path.isdir(os.path.join(root, "devices")):
            return "v1"
        if os.path.exists(os.path.join(root, "cgroup.controllers")):
            return "v2"
        # hybrid hosts mount the v1 devices controller; absent both, assume unified
        return "v2"

    def pod_dirs(self, pod: dict) -> List[str]:
        uid = uid_of(pod)
        qos = qos_class(pod)
        order = [qos] + [q for q in ("Guaranteed", QOS_BURSTABLE, QOS_BESTEFFORT) if q != qos]
        drivers = ("systemd", "cgroupfs") if self.driver == "auto" else (self.driver,)
        out = []
        for q in order:
            for d in drivers:
                if d == "systemd":
                    if q == QOS_BURSTABLE:
                        rel = f"kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{_esc(uid)}.slice"
                    elif q == QOS_BESTEFFORT:
                        rel = f"kubepods.slice/kubepods-besteffort.slice/kubepods-besteffort-pod{_esc(uid)}.slice"
                    else:
                        rel = f"kubepods.slice/kubepods-pod{_esc(uid)}.slice"
                else:
                    if q == QOS_BURSTABLE:
                        rel = f"kubepods/burstable/pod{uid}"
                    elif q == QOS_BESTEFFORT:
                        rel = f"kubepods/besteffort/pod{uid}"
                    else:
                        rel = f"kubepods/pod{uid}"
                out.append(os.path.join(self.base, rel))
        return out

    def container_dir(self, pod: dict, ctr: ContainerRef) -> str:
        key = (uid_of(pod), ctr.id)
        hit = self._cache.get(key)
        if hit and os.path.isdir(hit):
            return hit
        for pdir in self.pod_dirs(pod):
            if not os.path.isdir(pdir):
                continue
            for pre in RUNTIME_SCOPE_PREFIXES:
                for name in (f"{pre}{ctr.id}.scope", f"{pre}{ctr.id}"):
                    cand = os.path.join(pdir, name)
                    if os.path.isdir(cand):
                        self._cache[key] = cand
                        return cand
            # unknown naming scheme: any child dir containing the id
            for cand in glob.glob(os.path.join(pdir, f"*{ctr.id}*")):
                if os.path.isdir(cand):
                    self._cache[key] = cand
                    return cand
        found = self._from_proc(ctr.id)
        if found:
            self._cache[key] = found
            return found
        raise CgroupError(f"cgroup of container {ctr.name} ({ctr.id[:12]}) of pod "
                          f"{pod['metadata'].get('namespace')}/{pod['metadata'].get('name')} "
                          f"not found under {self.base}")

    def _from_proc(self, container_id: str) -> Optional[str]:
        """Last resort, runtime- and driver-agnostic: any process whose /proc/<pid>/cgroup names
        the container id tells us its cgroup path (v2 line ``0::/…``, v1 ``N:devices:/…``)."""
        try:
            pids = [d for d in os.listdir(self.proc_root) if d.isdigit()]
        except OSError:
            return None
        want_ctrl = "devices" if self.mode == "v1" else ""
        for pid in pids:
            try:
                with open(os.path.join(self.proc_root, pid, "cgroup")) as fh:
                    lines = fh.read().splitlines()
            except OSError:
                continue
            for line in lines:
                parts = line.split(":", 2)
                if len(parts) != 3 or container_id not in parts[2]:
                    continue
                ctrls = parts[1].split(",") if parts[1] else [""]
                if want_ctrl not in ctrls:
                    continue
                cand = os.path.join(self.base, parts[2].lstrip("/"))
                if os.path.isdir(cand):
                    return cand
        return None

    def forget(self, pod_uid: str) -> None:
        for k in [k for k in self._cache if k[0] == pod_uid]:
            del self._cache[k]

    @staticmethod
    def pids(cgdir: str, recursive: bool = True) -> List[int]:
        """PIDs in the cgroup (and, for v2 container scopes, its sub-cgroups)."""
        lib = _native.host()
        out: List[int] = []
        buf = (C.c_int32 * 4096)()
        n = C.c_int(0)
        stack = [cgdir]
        while stack:
            d = stack.pop()
            path = os.path.join(d, "cgroup.procs")
            rc = lib.gm_proc_read_pids(path.encode(), buf, 4096, C.byref(n))
            if rc < 0 and rc != -errno.ENOENT:      # ENOENT: not a cgroup directory
                raise CgroupError(f"read {path}: {os.strerror(-rc)}")
            if rc >= 0:
                out.extend(buf[:min(n.value, 4096)])
            if recursive:
                try:
                    with os.scandir(d) as it:
                        stack.extend(e.path for e in it if e.is_dir(follow_symlinks=False))
                except (FileNotFoundError, NotADirectoryError):
                    pass
        return sorted(set(out))


# ------------------------------------------------------------------------------ rules
def rules_for(nodes: Iterable[DeviceNode], allow: bool, access: str = "rw") -> List[_native.DevRule]:
    acc = 0
    if "r" in access:
        acc |= _native.GM_ACC_READ
    if "w" in access:
        acc |= _native.GM_ACC_WRITE
    if "m" in access:
        acc |= _native.GM_ACC_MKNOD
    return [_native.DevRule(b"c", acc, 1 if allow else 0, 0, n.major, n.minor) for n in nodes]


def _rule_array(rules: Sequence[_native.DevRule]):
    arr = (_native.DevRule * max(len(rules), 1))()
    for i, r in enumerate(rules):
        arr[i] = r
    return arr


def format_rule(r: _native.DevRule) -> str:
    buf = C.create_string_buffer(64)
    _native.host().gm_cg1_format_rule(C.byref(r), buf, 64)
    return buf.value.decode()


class DeviceRuleBackend(ABC):
    name = "abstract"

    @abstractmethod
    def apply(self, cgdir: str, grant: Sequence[DeviceNode], revoke: Sequence[DeviceNode],
              desired: Sequence[DeviceNode]) -> None:
        """Make ``grant`` accessible and ``revoke`` inaccessible. ``desired`` is the complete set
        of nodes gpumounter wants allowed after the call (full-state backends use it)."""

    @abstractmethod
    def allowed(self, cgdir: str) -> Set[Tuple[int, int]]:
        """(major, minor) pairs currently granted by gpumounter."""

    def installed(self, cgdir: str) -> Set[Tuple[int, int]]:
        """Pairs gpumounter's own installed state grants, whatever other parties' programs
        decide (:meth:`allowed` is the effective verdict). The journal forgets a rule only when
        it is gone from here — a foreign veto does not make a grant of ours go away."""
        return self.allowed(cgdir)

    def fingerprint(self, cgdir: str) -> object:
        """A cheap token of the cgroup's device-control state (one syscall or one small read):
        it changes whenever anyone — the runtime re-attaching its program, ``runc update``,
        systemd re-realising a unit, a write to devices.allow/deny — changes what the cgroup
        enforces. The device guard (worker/reconciler.py) compares it every second instead of
        re-auditing every hot container."""
        return None

    def prune(self) -> int:
        """Drop cached state of cgroups that no longer exist (containers gone without a detach);
        returns how many. Backends that cache nothing have nothing to drop."""
        cache = getattr(self, "_installed", None)
        if not cache:
            return 0
        gone = [d for d in cache if not os.path.isdir(d)]
        for d in gone:
            cache.pop(d, None)
        return len(gone)


V1_SYNC_STATE = ".gm_v1_applied"


def v1_fake_sync(cgdir: str) -> List[str]:
    """The kernel's side of an emulated v1 devices cgroup (one with ``FAKE_MARKER``): fold the
    ``devices.allow``/``devices.deny`` lines written since the last sync into the set of rules
    granted beyond the runtime's defaults, with the kernel's set semantics (an allow adds the
    rule, a deny removes it; both are idempotent), and return that set. Counting allow lines
    against deny lines, as the emulation did before, is not the kernel: a redundant deny
    (harmless on a real node) left a rule's count below zero and made the next allow read as
    missing. Lines that arrived on both files since the last sync are taken denies first, the
    order :meth:`V1Backend.apply` writes them in (it syncs after every call). A file that
    shrank was emptied by the emulation (a container's fresh device state): the set starts
    over. Serialised across processes by a lock on the state file."""
    import fcntl
    state = os.path.join(cgdir, V1_SYNC_STATE)
    try:
        fd = os.open(state, os.O_RDWR | os.O_CREAT, 0o644)
    except FileNotFoundError:
        return []                                # the cgroup is gone
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        raw = b""
        while True:
            chunk = os.read(fd, 65536)
            if not chunk:
                break
            raw += chunk
        try:
            st = json.loads(raw) if raw else {}
        except ValueError:
            st = {}
        rules: List[str] = st.get("rules", [])
        data = {}
        for name in ("deny", "allow"):
            try:
                with open(os.path.join(cgdir, f"devices.{name}"), "rb") as fh:
                    data[name] = fh.read()
            except FileNotFoundError:
                data[name] = b""
        if any(len(data[n]) < st.get(n, 0) for n in data):
            st, rules = {}, []
        new = {n: [ln.strip() for ln in data[n][st.get(n, 0):].decode().splitlines()
                   if ln.strip()] for n in data}
        if new["deny"] or new["allow"] or not raw:
            for rule in new["deny"]:
                rules = [r for r in rules if r != rule]
            for rule in new["allow"]:
                if rule not in rules:
                    rules.append(rule)
            os.lseek(fd, 0, os.SEEK_SET)
            os.ftruncate(fd, 0)
            os.write(fd, json.dumps({"deny": len(data["deny"]), "allow": len(data["allow"]),
                                     "rules": rules}).encode())
        return rules
    finally:
        os.close(fd)


class V1Backend(DeviceRuleBackend):
    name = "cgroup-v1"

    def apply(self, cgdir, grant, revoke, desired):
        rules = rules_for(revoke, allow=False) + rules_for(grant, allow=True)
        if not rules:
            return
        if _log.isEnabledFor(10):
            _log.debug("devices rules in %s: deny %s allow %s", cgdir,
                       sorted((n.major, n.minor) for n in revoke),
                       sorted((n.major, n.minor) for n in grant))
        rc = _native.host().gm_cg1_apply(cgdir.encode(), _rule_array(rules), len(rules))
        if rc < 0:
            raise CgroupError(f"devices.allow/deny write in {cgdir}: {os.strerror(-rc)}")
        if os.path.exists(os.path.join(cgdir, FAKE_MARKER)):
            v1_fake_sync(cgdir)          # an emulated cgroup: the kernel's part, in write order

    def fingerprint(self, cgdir):
        if os.path.exists(os.path.join(cgdir, FAKE_MARKER)):
            names = ("devices.allow", "devices.deny")
        else:
            names = ("devices.list",)
        out = []
        for fname in names:
            try:
                with open(os.path.join(cgdir, fname), "rb") as fh:
                    out.append(fh.read())
            except OSError:
                out.append(None)
        return tuple(out)

    def allowed(self, cgdir):
        if os.path.exists(os.path.join(cgdir, FAKE_MARKER)):
            out = set()                  # writes by others (a test, the runtime) land first
            for rule in v1_fake_sync(cgdir):
                parts = rule.split()
                if len(parts) == 3 and parts[0] == "c" and "*" not in parts[1]:
                    ma, mi = parts[1].split(":")
                    out.add((int(ma), int(mi)))
            return out
        out = set()
        try:
            with open(os.path.join(cgdir, "devices.list")) as fh:
                for line in fh:
                    parts = line.split()
                    if len(parts) == 3 and parts[0] == "c" and "*" not in parts[1]:
                        ma, mi = parts[1].split(":")
                        out.add((int(ma), int(mi)))
        except FileNotFoundError:
            pass
        return out


# OCI/runc default device allow-list, compiled into our program only if the tail-call chain to
# the runtime's own program was lost (unpinned map + worker restart).
OCI_DEFAULT_RULES = [("c", 1, -1, -1), ("b", 1, -1, -1), ("c", 7, 1, 3), ("c", 7, 1, 5),
                     ("c", 7, 1, 7), ("c", 7, 1, 8), ("c", 7, 1, 9), ("c", 7, 5, 0),
                     ("c", 7, 5, 1), ("c", 7, 5, 2), ("c", 7, 136, -1), ("c", 7, 10, 200)]


def oci_default_rules() -> List[_native.DevRule]:
    return [_native.DevRule(t.encode(), acc, 1, 0, ma, mi) for t, acc, ma, mi in OCI_DEFAULT_RULES]


class V2BpfBackend(DeviceRuleBackend):
    """Real eBPF backend (needs CAP_SYS_ADMIN + CAP_BPF on a cgroup2 mount).

    ``pin_dir`` is a directory on a bpffs (``/sys/fs/bpf/gpumounter`` in the DaemonSet) where the
    tail-call map to the runtime's program is pinned so the chain survives worker restarts.
    """

    name = "cgroup-v2-bpf"

    def __init__(self, pin_dir: str = "", set_mode: bool = True) -> None:
        self.pin_dir = pin_dir
        if pin_dir:
            os.makedirs(pin_dir, exist_ok=True)
        # set mode (default): rules in an allow-set map; False = straight-line programs (the
        # native switch is process-wide; a worker has one backend)
        self.set_mode = set_mode
        _native.host().gm_bpf_dev_straight_line(0 if set_mode else 1)
        # cgroup → (attached program ids, pairs those programs grant), recorded when this
        # process installed them. Program ids are kernel-unique while a program is loaded and
        # a loaded program's instructions are immutable, so while the cgroup's attached id list
        # is exactly this tuple the kernel enforces what we built — :meth:`allowed` then skips
        # reading back and interpreting the xlated code (the attach verify step). Any other id
        # list (systemd or the runtime swapped a program, a foreign one joined) takes the full
        # read-back path.
        self._installed: Dict[str, Tuple[Tuple[int, ...], FrozenSet[Tuple[int, int]]]] = {}

    def sweep_pins(self, cgroup_root: str) -> List[str]:
        """Unpin the tail-call maps of cgroups that no longer exist (``gm_<cgroup inode>_<id>``
        under ``pin_dir``). A container that exits while it holds hot-mounted GPUs takes its
        cgroup and our attached program with it, but the pinned map would live on — and keep
        the runtime's program it chains to loaded. Live inodes come from one walk of the cgroup
        tree (readdir's d_ino, no stat per directory). Returns the names removed."""
        if not self.pin_dir or not os.path.isdir(self.pin_dir):
            return []
        pins = [f for f in os.listdir(self.pin_dir) if f.startswith("gm_")]
        if not pins:
            return []
        live = set()
        try:
            live.add(os.stat(cgroup_root).st_ino)
        except OSError:
            return []              # cannot see the hierarchy: judge nothing
        stack = [cgroup_root]
        while stack:
            d = stack.pop()
            try:
                with os.scandir(d) as it:
                    for e in it:
                        if e.is_dir(follow_symlinks=False):
                            live.add(e.inode())
                            stack.append(e.path)
            except OSError:
                continue           # removed while walking
        removed = []
        for f in pins:
            parts = f.split("_")
            try:
                ino = int(parts[1])
            except (IndexError, ValueError):
                continue
            if ino not in live:
                try:
                    os.unlink(os.path.join(self.pin_dir, f))
                    removed.append(f)
                except FileNotFoundError:
                    pass
        if removed:
            log.kv(_log, 20, "unpinned chain maps of removed cgroups", maps=removed)
        return removed

    @staticmethod
    def attached_ids(cgdir: str) -> Tuple[int, ...]:
        ids, n, flags = (C.c_uint32 * 16)(), C.c_uint32(0), C.c_uint32(0)
        rc = _native.host().gm_bpf_dev_query(cgdir.encode(), ids, 16, C.byref(n), C.byref(flags))
        if rc < 0:
            raise CgroupError(f"bpf query on {cgdir}: {os.strerror(-rc)}")
        return tuple(int(ids[i]) for i in range(min(n.value, 16)))

    def fingerprint(self, cgdir):
        # the attached program ids (BPF_PROG_QUERY): a swapped or added program changes them;
        # the set-mode allow map changes only through us
        try:
            return self.attached_ids(cgdir)
        except CgroupError:
            return None

    def apply(self, cgdir, grant, revoke, desired):
        lib = _native.host()
        pin = self.pin_dir.encode() if self.pin_dir else None
        self._installed.pop(cgdir, None)
        if not desired:
            rc = lib.gm_bpf_dev_restore(cgdir.encode(), pin)
            if rc < 0:
                raise CgroupError(f"bpf restore on {cgdir}: {os.strerror(-rc)}")
            return
        rules = rules_for(desired, allow=True)
        base = oci_default_rules()
        pid, chained = C.c_uint32(0), C.c_uint32(0)
        rc = lib.gm_bpf_dev_install(cgdir.encode(), _rule_array(rules), len(rules),
                                    _rule_array(base), len(base), pin, C.byref(pid),
                                    C.byref(chained))
        if rc < 0:
            raise CgroupError(f"bpf install on {cgdir}: {os.strerror(-rc)}")
        if not self.set_mode and rc == 1 and pid.value:
            # one slot: our straight-line program replaced the runtime's in place
            self._installed[cgdir] = ((pid.value,),
                                      frozenset((n.major, n.minor) for n in desired))
        # set mode: the kernel's map is the record, read back by allowed()
        if trace.current() is not None:
            tm = _native.BpfTiming()
            lib.gm_bpf_dev_last_timing(C.byref(tm))
            trace.record("bpf_query", tm.query_ns)
            trace.record("bpf_build", tm.build_ns, insns=tm.insns)
            trace.record("bpf_load_verify", tm.load_ns, programs=tm.programs)
            trace.record("bpf_chain_map", tm.map_ns)
            trace.record("bpf_attach", tm.attach_ns)
        log.kv(_log, 10, "bpf program installed", cgroup=cgdir, prog_id=pid.value,
               chained=chained.value, rules=len(rules))

    def allowed(self, cgdir):
        """What the kernel enforces, read back from it: for a set-mode program of ours the
        contents of its allow-set map (one native call); for a straight-line one its xlated
        instructions, evaluated by the interpreter. A pair counts only if every program of ours
        grants it. A program that systemd or the runtime swapped out reads as "nothing granted",
        so the reconciler re-installs it. A foreign program attached next to ours (systemd
        re-realising its unit) can veto any access under BPF_F_ALLOW_MULTI, so its own verdict
        is evaluated too: with the unit's DeviceAllow= kept in step (node/systemd.py) it grants
        our nodes; otherwise the pair reads as missing and the re-install wraps that program.

        Fast path for straight-line programs: when the attached id list is exactly the one this
        backend installed, the answer is the rule set it compiled into that program (programs
        are immutable; see ``_installed``). Set-mode programs keep their id while their map
        changes, so their set is always read."""
        known = self._installed.get(cgdir)
        if known is not None:
            try:
                if self.attached_ids(cgdir) == known[0]:
                    return set(known[1])
            except CgroupError:
                pass
            self._installed.pop(cgdir, None)
        out = self.installed(cgdir)
        foreign = _program_at(cgdir, 0, foreign_only=True)[1] if out else 0
        for i in range(foreign):
            prog, _ = _program_at(cgdir, i, foreign_only=True)
            if prog is None:
                break
            try:
                out = bpfvm.allowed_pairs(prog, sorted(out), chained=lambda *a: 0)
            except bpfvm.BpfError:
                return set()                   # cannot judge it: assume it vetoes
        return out

    def installed(self, cgdir):
        """What gpumounter's own attached programs grant together (each must allow a pair),
        before any foreign program's verdict."""
        grants: List[Set[Tuple[int, int]]] = []
        while True:
            kind, pairs = _set_at(cgdir, len(grants))
            if kind is None:
                break
            if kind == "code":
                prog, _ = _program_at(cgdir, len(grants))
                pairs = program_allows(prog) if prog is not None else set()
            grants.append(pairs)
        if not grants:
            return set()
        out = grants[0]
        for g in grants[1:]:
            out &= g
        return out


def _set_at(cgdir: str, index: int):
    """("set", rw char pairs) for a set-mode program of ours at ``index``, ("code", None) for a
    straight-line one, (None, None) past the last."""
    lib = _native.host()
    cap = 64
    while True:
        ent = (C.c_uint32 * (4 * cap))()
        n, pid = C.c_uint32(0), C.c_uint32(0)
        rc = lib.gm_bpf_dev_set_at(cgdir.encode(), index, ent, cap, C.byref(n), C.byref(pid))
        if rc == -errno.ENOSPC:
            cap = n.value + 16
            continue
        break
    if rc == -errno.ENOENT:
        return None, None
    if rc < 0:
        raise CgroupError(f"bpf allow-set read-back on {cgdir}: {os.strerror(-rc)}")
    if rc == 0:
        return "code", None
    rw = bpfvm.ACC_READ | bpfvm.ACC_WRITE
    return "set", {(int(ent[4 * i + 1]), int(ent[4 * i + 2])) for i in range(n.value)
                   if ent[4 * i] == bpfvm.BPF_DEVCG_DEV_CHAR and (ent[4 * i + 3] & rw) == rw}


def _program_at(cgdir: str, index: int, foreign_only: bool = False
                ) -> Tuple[Optional[List[int]], int]:
    lib = _native.host()
    n, pid, foreign = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    fo = 1 if foreign_only else 0
    rc = lib.gm_bpf_dev_program_at(cgdir.encode(), index, fo, None, 0, C.byref(n), C.byref(pid),
                                   C.byref(foreign))
    if rc == 0 and n.value == 0:
        return None, foreign.value
    if rc not in (0, -errno.ENOSPC):
        raise CgroupError(f"bpf introspection on {cgdir}: {os.strerror(-rc)}")
    buf = (C.c_uint64 * n.value)()
    rc = lib.gm_bpf_dev_program_at(cgdir.encode(), index, fo, buf, n.value, C.byref(n),
                                   C.byref(pid), C.byref(foreign))
    if rc < 0:
        raise CgroupError(f"bpf introspection on {cgdir}: {os.strerror(-rc)}")
    return [int(buf[i]) for i in range(n.value)], foreign.value


def attached_programs(cgdir: str) -> Tuple[List[List[int]], int]:
    """(xlated instructions of each gpumounter program, number of foreign programs) attached."""
    progs: List[List[int]] = []
    foreign = 0
    while True:
        prog, foreign = _program_at(cgdir, len(progs))
        if prog is None:
            return progs, foreign
        progs.append(prog)


def attached_program(cgdir: str) -> Optional[List[int]]:
    progs, _ = attached_programs(cgdir)
    return progs[0] if progs else None


def program_allows(prog: Sequence[int]) -> Set[Tuple[int, int]]:
    """(major, minor) pairs a device program grants for rw char access, over every constant it
    compares against; the chained runtime program is modelled by runc's default list. A pure
    function of the instruction words, so the interpretation is memoised on them (the program
    itself is still read back from the kernel on every call); callers get their own copy."""
    return set(_program_allows(tuple(prog)))


@functools.lru_cache(maxsize=256)
def _program_allows(prog: Tuple[int, ...]) -> FrozenSet[Tuple[int, int]]:
    consts = bpfvm.immediates(list(prog))
    return frozenset(bpfvm.allowed_pairs(list(prog), [(a, b) for a in consts for b in consts]))


@functools.lru_cache(maxsize=4)
def _set_program_words(chained: bool = True) -> Tuple[int, ...]:
    return tuple(build_set_program(chained))


def build_set_program(chained: bool) -> List[int]:
    """The set-mode program (gm_bpf_dev_build_set) with placeholder map fds (0): the allow-set
    map is ``maps={0: ...}`` for :func:`bpfvm.run`."""
    lib = _native.host()
    ch = -2 if chained else -1
    need = -lib.gm_bpf_dev_build_set(-2, None, 0, 0 if chained else 1, ch, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build_set(-2, None, 0, 0 if chained else 1, ch, buf, need)
    if n < 0:
        raise CgroupError("bpf set program build failed")
    return [int(buf[i]) for i in range(n)]


def build_program(nodes: Sequence[DeviceNode], chained: bool) -> List[int]:
    rules = rules_for(nodes, allow=True)
    lib = _native.host()
    need = -lib.gm_bpf_dev_build(_rule_array(rules), len(rules), 0 if chained else 1,
                                 -2 if chained else -1, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build(_rule_array(rules), len(rules), 0 if chained else 1,
                             -2 if chained else -1, buf, need)
    if n < 0:
        raise CgroupError("bpf program build failed")
    return [int(buf[i]) for i in range(n)]


class V2RecordingBackend(DeviceRuleBackend):
    """Builds the exact program the v2 backend would load and records it beside the cgroup."""

    name = "cgroup-v2-recording"

    def apply(self, cgdir, grant, revoke, desired):
        path = os.path.join(cgdir, BPF_STATE)
        self._installed.pop(cgdir, None)
        if not desired:
            if os.path.exists(path):
                os.unlink(path)
            return
        # what V2BpfBackend installs: the set-mode program and its allow-set map
        state = {"rules": [[n.major, n.minor, n.path] for n in desired],
                 "chained": "runtime-default", "mode": "set",
                 "set": [[bpfvm.BPF_DEVCG_DEV_CHAR, n.major, n.minor,
                          bpfvm.ACC_READ | bpfvm.ACC_WRITE] for n in desired],
                 "insns": [f"{i:016x}" for i in _set_program_words()]}
        blob = json.dumps(state).encode()
        tmp = path + ".tmp"
        with open(tmp, "wb") as fh:
            fh.write(blob)
        os.replace(tmp, path)  # atomic like BPF_F_REPLACE
        # the recorded file stands in for the attached program, and its exact bytes play the
        # role of the program id in V2BpfBackend's fast path (stat metadata would not do: the
        # rename reuses inode numbers and rewrites within one tick share an mtime)
        self._installed[cgdir] = (blob, frozenset((n.major, n.minor) for n in desired))

    def __init__(self) -> None:
        self._installed: Dict[str, Tuple[bytes, FrozenSet[Tuple[int, int]]]] = {}

    def fingerprint(self, cgdir):
        try:
            with open(os.path.join(cgdir, BPF_STATE), "rb") as fh:
                return fh.read()
        except OSError:
            return None

    def allowed(self, cgdir):
        path = os.path.join(cgdir, BPF_STATE)
        try:
            with open(path, "rb") as fh:
                blob = fh.read()
        except FileNotFoundError:
            self._installed.pop(cgdir, None)
            return set()
        known = self._installed.get(cgdir)
        if known is not None and known[0] == blob:
            return set(known[1])
        st = json.loads(blob)
        prog = [int(x, 16) for x in st["insns"]]
        if st.get("mode") != "set":       # recorded by an older worker: a straight-line program
            return program_allows(prog)
        # evaluate the recorded program against its recorded map (the runtime's program, which
        # it tail-calls, is not consulted: only what gpumounter grants counts)
        table = {(t, ma, mi): acc for t, ma, mi, acc in st["set"]}
        return bpfvm.allowed_pairs(prog, sorted({(k[1], k[2]) for k in table}),
                                   chained=lambda *a: 0, maps={0: table})


def make_backend(mode: str, emulate: bool, bpf_pin_dir: str = "",
                 bpf_set_mode: bool = True) -> DeviceRuleBackend:
    if mode == "v1":
        return V1Backend()
    if emulate:
        return V2RecordingBackend()
    return V2BpfBackend(bpf_pin_dir, bpf_set_mode)
