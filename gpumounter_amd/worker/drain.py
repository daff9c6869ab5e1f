"""Placeholders that keep a force-removed GPU booked until the killed processes are gone.

The reference's force removal runs deny → rm → kill (SIGTERM) and then deletes the slave pods
with the default delete options, polling until they are NotFound (reference:
pkg/util/util.go:112-143, pkg/util/gpu/allocator/allocator.go:128-156,284-317): the GPU stays in
the scheduler's books through the slave's termination grace. A device-cgroup revoke only gates
``open()``; a process that already holds ``/dev/kfd`` and a render node keeps using the GPU
until it exits. So here the placeholder is released only once every killed process has exited
(pidfd readable). A process that survives SIGKILL for ``kill_reap_s`` (uninterruptible sleep in
the driver) leaves its placeholder *draining*:

* it is detached from the tenant (owner labels, ownerReference and UID annotation removed), so
  the tenant's mount state no longer includes the GPU and nothing re-grants it;
* it keeps its ledger entry, so neither the scheduler nor another attach can take the GPU;
* ``gpumounter.amd.com/drain-pids`` records ``pid:starttime`` of every process waited on, so a
  restarted worker (which holds no pidfds) still knows exactly which processes to wait for;
* this worker waits on the pidfds (event-driven, no polling) and releases the placeholder the
  moment the last one exits; the reconciler's sweep covers the restart case.

Marking is a PATCH, and it can fail. Until it succeeds the placeholder is *unmarked*: still
labelled as the tenant's, but its GPU's access is already revoked, so it is left out of the
tenant's mount state (nothing re-grants it, RemoveGPU does not offer it again) and is never
released while a killed process runs. The mark is retried (0.1/0.5/2/5/15 s, then every 30 s)
alongside the pidfd wait; the pending set is kept in ``<state_dir>/drain_pending.json`` so a
restarted worker resumes it (by ``pid:starttime``) instead of re-granting the GPU.
"""
from __future__ import annotations

import asyncio
import json
import os
from typing import Dict, List, Sequence, Tuple

from gpumounter_amd.cluster.kube import NotFound
from gpumounter_amd.cluster.placeholder import Placeholder
from gpumounter_amd.models.types import (ANN_DRAIN_OWNER, ANN_DRAIN_PIDS, ANN_GROUP,
                                         ANN_IDEMPOTENCY, ANN_MOUNT_MODE, ANN_OWNER_UID,
                                         LABEL_OWNER, LABEL_OWNER_NS, MODE_DRAINING)
from gpumounter_amd.models import pod as podu
from gpumounter_amd.node import procs
from gpumounter_amd.utils import log

_log = log.get("worker.drain")


def is_draining(p: dict) -> bool:
    return (p["metadata"].get("annotations") or {}).get(ANN_MOUNT_MODE) == MODE_DRAINING


def parse_pids(value: str) -> List[Tuple[int, int]]:
    out = []
    for item in (value or "").split(","):
        pid, _, started = item.partition(":")
        try:
            out.append((int(pid), int(started or 0)))
        except ValueError:
            continue
    return out


class DrainKeeper:
    # a failed draining mark is retried after these delays, then every MARK_RETRY_LAST_S
    MARK_RETRY_S = (0.1, 0.5, 2.0, 5.0, 15.0)
    MARK_RETRY_LAST_S = 30.0

    def __init__(self, service) -> None:
        self.svc = service
        # placeholder uid → (placeholder, the pidfds still waited on)
        self.held: Dict[str, Tuple[Placeholder, procs.Pinned]] = {}
        # placeholder uid → {"ns", "name", "owner", "pids"}: revoked from its tenant, still
        # booked, draining mark not written yet (retried; persisted for a restarted worker)
        self.unmarked: Dict[str, dict] = {}
        sd = getattr(getattr(service, "cfg", None), "state_dir", "")
        self._path = os.path.join(sd, "drain_pending.json") if sd else ""
        self._load()
        self._tasks: set = set()
        self.released = 0

    # ------------------------------------------------------------------------ pending marks
    def _load(self) -> None:
        if not self._path:
            return
        try:
            with open(self._path, encoding="utf-8") as fh:
                self.unmarked = {k: v for k, v in json.load(fh).items() if isinstance(v, dict)}
        except FileNotFoundError:
            pass
        except (OSError, ValueError) as e:
            _log.error("drain: unreadable %s (%s); ignoring it", self._path, e)

    def _save(self) -> None:
        if not self._path:
            return
        tmp = self._path + ".tmp"
        try:
            os.makedirs(os.path.dirname(self._path), mode=0o700, exist_ok=True)
            with open(tmp, "w", encoding="utf-8") as fh:
                fh.write(json.dumps(self.unmarked))
            os.replace(tmp, self._path)
        except OSError as e:
            _log.error("drain: cannot persist pending marks: %s", e)

    def _patch(self, owner: str, mark: str) -> dict:
        return {"metadata": {
            "labels": {LABEL_OWNER: None, LABEL_OWNER_NS: None},
            "ownerReferences": None,
            "annotations": {ANN_MOUNT_MODE: MODE_DRAINING, ANN_DRAIN_PIDS: mark,
                            ANN_DRAIN_OWNER: owner, ANN_OWNER_UID: None, ANN_IDEMPOTENCY: None,
                            ANN_GROUP: None}}}

    async def _mark(self, phs: Sequence[Placeholder], owner: str, mark: str
                    ) -> List[Placeholder]:
        """PATCH ``phs`` into draining placeholders; returns those not marked (they stay in
        :attr:`unmarked`, persisted)."""
        kube = self.svc.ph.kube
        epoch = self.svc.ph.informer.epoch
        patch = self._patch(owner, mark)
        res = await asyncio.gather(*[kube.patch_pod(p.namespace, p.name, patch) for p in phs],
                                   return_exceptions=True)
        failed = []
        for ph, r in zip(phs, res):
            if isinstance(r, dict):
                self.svc.ph.informer.upsert(r, epoch)
                ph.mode = MODE_DRAINING
                ph.owner_uid = ""                       # the mark removes the owner
                self.unmarked.pop(ph.uid, None)
            elif isinstance(r, NotFound):
                self.unmarked.pop(ph.uid, None)     # gone: nothing left to book
            else:
                _log.error("mark %s/%s draining: %s (retried)", ph.namespace, ph.name, r)
                self.unmarked[ph.uid] = {"ns": ph.namespace, "name": ph.name, "owner": owner,
                                         "pids": mark}
                failed.append(ph)
        self._save()
        return failed

    def _delays(self):
        yield from self.MARK_RETRY_S
        while True:
            yield self.MARK_RETRY_LAST_S

    # ------------------------------------------------------------------------ hold / wait
    async def hold(self, owner: dict, phs: Sequence[Placeholder], pinned: procs.Pinned,
                   pids: Sequence[int]) -> List[Placeholder]:
        """Turn ``phs`` into draining placeholders waiting for ``pids`` (taking ownership of
        ``pinned``). Returns the placeholders whose mark failed: they are revoked and booked
        all the same, and the mark is retried until it lands or the processes are gone."""
        pinned.keep_only(pids)
        mark = ",".join(f"{p}:{procs.start_time(p)}" for p in sorted(pids))
        who = f"{podu.ns_of(owner)}/{podu.name_of(owner)}"
        failed = await self._mark(phs, who, mark)
        for ph in phs:
            self.held[ph.uid] = (ph, pinned)
        self.svc.metrics.draining.set(len(self.held))
        self.svc.metrics.reconcile_actions.labels(action="drain_hold").inc(len(phs))
        log.kv(_log, 30, "GPU held until killed processes exit", pids=list(pids),
               placeholders=[p.name for p in phs], unmarked=[p.name for p in failed])
        t = asyncio.ensure_future(self._wait(list(phs), pinned, list(pids), who, mark))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return failed

    async def _wait(self, phs: List[Placeholder], pinned: procs.Pinned, pids: List[int],
                    owner: str, mark: str) -> None:
        delays = self._delays()
        try:
            while pinned.fds:
                pending = [ph for ph in phs if ph.uid in self.unmarked]
                left = await pinned.wait_exit(pids, next(delays) if pending else 3600.0)
                if not left:
                    break
                if pending:
                    await self._mark(pending, owner, mark)
            pinned.close()
            await self._release(phs)
        except asyncio.CancelledError:
            pinned.close()
            raise
        except Exception as e:  # noqa: BLE001 - the reconciler's sweep retries the release
            _log.error("drain release failed: %s", e)

    async def resume(self) -> None:
        """Worker start-up: marks a previous worker could not write. A placeholder still there
        is marked (or released once its recorded processes are gone), retried in the
        background; one gone is forgotten."""
        for uid, rec in list(self.unmarked.items()):
            cur = self.svc.ph.informer.cache.get((rec.get("ns"), rec.get("name")))
            if cur is None or cur["metadata"].get("uid") != uid:
                self.unmarked.pop(uid, None)
                continue
            t = asyncio.ensure_future(self._resume_one(uid, rec))
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)
        self._save()

    async def _resume_one(self, uid: str, rec: dict) -> None:
        cur = self.svc.ph.informer.cache.get((rec["ns"], rec["name"])) or {"metadata": {}}
        # unmarked: it still names the Pod it was removed from as its owner
        ph = Placeholder(rec["ns"], rec["name"], uid, owner_uid=(
            cur["metadata"].get("annotations") or {}).get(ANN_OWNER_UID) or "")
        delays = self._delays()
        while uid in self.unmarked:
            if not any(procs.same_process(pid, st) for pid, st in parse_pids(rec["pids"])):
                try:
                    await self._release([ph])
                except Exception as e:  # noqa: BLE001 - retried below
                    _log.error("drain release failed: %s", e)
                else:
                    return
            else:
                await self._mark([ph], rec["owner"], rec["pids"])
            if uid in self.unmarked:
                await asyncio.sleep(next(delays))

    async def _release(self, phs: Sequence[Placeholder]) -> None:
        for ph in phs:
            self.held.pop(ph.uid, None)
        self.svc.metrics.draining.set(len(self.held))
        await self.svc.ph.release(list(phs))
        if any(self.unmarked.pop(ph.uid, None) is not None for ph in phs):
            self._save()
        self.released += len(phs)
        self.svc.metrics.reconcile_actions.labels(action="drain_release").inc(len(phs))
        log.kv(_log, 20, "drained GPU released", placeholders=[p.name for p in phs])

    async def sweep(self) -> List[str]:
        """Draining placeholders this worker holds no pidfds for (it restarted): release those
        whose recorded processes have all exited. (PID, start time) identifies each process,
        so a recycled PID never keeps a GPU booked, nor does it release one early."""
        out = []
        for p in self.svc.ph.live():
            if not is_draining(p):
                continue
            md = p["metadata"]
            if md.get("uid") in self.held:
                continue
            waits = parse_pids((md.get("annotations") or {}).get(ANN_DRAIN_PIDS, ""))
            if any(procs.same_process(pid, st) for pid, st in waits):
                continue
            ph = self.svc.ph.cached(p) or self.svc.ph.from_pod(p, {})
            try:
                await self._release([ph])
            except NotFound:
                pass
            out.append(md["name"])
        return out

    def waiting(self) -> Dict[str, List[int]]:
        return {ph.name: pin.pids() for ph, pin in self.held.values()}

    async def stop(self) -> None:
        for t in list(self._tasks):
            t.cancel()
        for t in list(self._tasks):
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        for _, pin in list(self.held.values()):
            pin.close()
        self.held.clear()
