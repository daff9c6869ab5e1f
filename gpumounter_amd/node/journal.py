"""Node-local injection journal: exactly which device rules and nodes gpumounter put into which
container, keyed by container ID.

The reference only ever revokes what its ledger assigns to the pod it was asked about — it denies,
unlinks and kills for the GPUs ``GetRemoveGPU`` selects (reference: pkg/util/util.go:73-147,
selection at pkg/util/gpu/allocator/allocator.go:101-126) and never sweeps other pods. The
reconciler here does sweep (it repairs drift the reference leaves behind), so it needs
a record of what it owns: a GPU node or rule found in a container is only ever revoked when this
journal says gpumounter created it. Device nodes a container already had (privileged pods, pods
that mount the host's ``/dev``, device-plugin GPUs, a node the image ships) are never recorded and
therefore never touched.

Write-ahead protocol (:class:`~gpumounter_amd.node.hotmount.HotMount`):

* before granting/creating, the *intended* rules/nodes are recorded (:meth:`intend`), so a worker
  that dies between the kernel call and the bookkeeping still knows the state is its own;
* after creating, nodes that turned out to exist already are dropped again (:meth:`settle`), so a
  pre-existing node is never later unlinked;
* after revoking/unlinking, the entries are removed (:meth:`forget`).

Storage: one small JSON file per container under ``state_dir`` (a hostPath in the DaemonSet,
``/var/lib/gpumounter/journal``), replaced atomically with ``rename(2)``. No ``fsync``: the record
only has to survive a worker crash (the page cache does), and a node crash takes every container —
and so every cgroup rule and ``/dev`` it describes — down with it. ``state_dir=""`` keeps the journal
in memory only (unit tests).
"""
from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Tuple

from gpumounter_amd.utils import log

_log = log.get("node.journal")

Key = Tuple[int, int]


@dataclass
class Entry:
    container_id: str
    namespace: str = ""
    pod: str = ""
    pod_uid: str = ""
    container: str = ""
    cgdir: str = ""
    rules: Dict[Key, str] = field(default_factory=dict)   # (major, minor) → node path
    nodes: Dict[Key, str] = field(default_factory=dict)
    updated: float = 0.0

    def empty(self) -> bool:
        return not self.rules and not self.nodes

    def to_json(self) -> dict:
        return {"container_id": self.container_id, "namespace": self.namespace, "pod": self.pod,
                "pod_uid": self.pod_uid, "container": self.container, "cgdir": self.cgdir,
                "rules": sorted([ma, mi, p] for (ma, mi), p in self.rules.items()),
                "nodes": sorted([ma, mi, p] for (ma, mi), p in self.nodes.items()),
                "updated": self.updated}

    @classmethod
    def from_json(cls, d: dict) -> "Entry":
        return cls(d["container_id"], d.get("namespace", ""), d.get("pod", ""),
                   d.get("pod_uid", ""), d.get("container", ""), d.get("cgdir", ""),
                   {(int(a), int(b)): p for a, b, p in d.get("rules", [])},
                   {(int(a), int(b)): p for a, b, p in d.get("nodes", [])},
                   float(d.get("updated", 0.0)))


def _safe_id(cid: str) -> bool:
    return bool(cid) and all(c.isalnum() or c in "-_." for c in cid) and cid[0] != "."


class InjectionJournal:
    def __init__(self, state_dir: str = "") -> None:
        self.dir = state_dir
        self._entries: Dict[str, Entry] = {}
        self._mu = threading.Lock()
        self.writes = 0
        if state_dir:
            os.makedirs(state_dir, mode=0o700, exist_ok=True)
            self._load()

    # ------------------------------------------------------------------------ persistence
    def _path(self, cid: str) -> str:
        return os.path.join(self.dir, cid + ".json")

    def _load(self) -> None:
        for fn in os.listdir(self.dir):
            if not fn.endswith(".json"):
                continue
            try:
                with open(os.path.join(self.dir, fn), encoding="utf-8") as fh:
                    e = Entry.from_json(json.load(fh))
            except (OSError, ValueError, KeyError, TypeError) as ex:
                _log.error("journal: unreadable record %s (%s); ignoring it", fn, ex)
                continue
            if e.container_id + ".json" == fn:
                self._entries[e.container_id] = e

    def _store(self, e: Entry) -> None:
        self.writes += 1
        if not self.dir:
            return
        path = self._path(e.container_id)
        if e.empty():
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass
            return
        tmp = path + ".tmp"
        # dumps (the C encoder) + one write(2): json.dump streams through the pure-Python
        # encoder, and a text file object costs more than the write itself on the attach path
        blob = json.dumps(e.to_json(), separators=(",", ":")).encode()
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_CLOEXEC, 0o600)
        try:
            view = memoryview(blob)
            while view:
                view = view[os.write(fd, view):]
        finally:
            os.close(fd)
        os.replace(tmp, path)

    # ------------------------------------------------------------------------ queries
    def get(self, cid: str) -> Optional[Entry]:
        return self._entries.get(cid)

    def entries(self) -> List[Entry]:
        with self._mu:
            return list(self._entries.values())

    def rules_of(self, cid: str) -> Dict[Key, str]:
        e = self._entries.get(cid)
        return dict(e.rules) if e else {}

    def nodes_of(self, cid: str) -> Dict[Key, str]:
        e = self._entries.get(cid)
        return dict(e.nodes) if e else {}

    def __len__(self) -> int:
        return sum(1 for e in self._entries.values() if not e.empty())

    # ------------------------------------------------------------------------ updates
    def _entry(self, cid: str, owner: Optional[dict]) -> Entry:
        if not _safe_id(cid):
            raise ValueError(f"journal: bad container id {cid!r}")
        e = self._entries.get(cid)
        if e is None:
            e = self._entries[cid] = Entry(cid)
        if owner:
            for k, v in owner.items():
                if v:
                    setattr(e, k, v)
        return e

    def intend(self, cid: str, rules: Iterable[Tuple[Key, str]] = (),
               nodes: Iterable[Tuple[Key, str]] = (), **owner: str) -> None:
        """Record rules/nodes about to be granted/created (write-ahead)."""
        with self._mu:
            e = self._entry(cid, owner)
            before = (len(e.rules), len(e.nodes))
            e.rules.update(rules)
            e.nodes.update(nodes)
            if (len(e.rules), len(e.nodes)) != before or not e.updated:
                e.updated = time.time()
                self._store(e)

    def settle(self, cid: str, not_ours: Iterable[Key]) -> None:
        """Drop nodes that existed before gpumounter's create call (never ours to unlink)."""
        keys = list(not_ours)
        if not keys:
            return
        with self._mu:
            e = self._entries.get(cid)
            if e is None:
                return
            changed = False
            for k in keys:
                changed |= e.nodes.pop(k, None) is not None
            if changed:
                e.updated = time.time()
                self._store(e)

    def forget(self, cid: str, rules: Iterable[Key] = (), nodes: Iterable[Key] = ()) -> None:
        with self._mu:
            e = self._entries.get(cid)
            if e is None:
                return
            changed = False
            for k in rules:
                changed |= e.rules.pop(k, None) is not None
            for k in nodes:
                changed |= e.nodes.pop(k, None) is not None
            if changed:
                e.updated = time.time()
                self._store(e)
            if e.empty():
                del self._entries[cid]

    def drop(self, cid: str) -> None:
        """The container is gone (its cgroup and mount namespace with it): nothing to revoke."""
        with self._mu:
            e = self._entries.pop(cid, None)
            if e is not None:
                e.rules.clear()
                e.nodes.clear()
                self._store(e)
