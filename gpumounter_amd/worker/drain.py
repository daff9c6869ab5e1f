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
"""
from __future__ import annotations

import asyncio
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
    def __init__(self, service) -> None:
        self.svc = service
        # placeholder uid → (placeholder, the pidfds still waited on)
        self.held: Dict[str, Tuple[Placeholder, procs.Pinned]] = {}
        self._tasks: set = set()
        self.released = 0

    async def hold(self, owner: dict, phs: Sequence[Placeholder], pinned: procs.Pinned,
                   pids: Sequence[int]) -> List[Placeholder]:
        """Turn ``phs`` into draining placeholders waiting for ``pids`` (taking ownership of
        ``pinned``). Returns the placeholders that could not be marked (the caller keeps them
        owned by the tenant, so they stay booked either way)."""
        pinned.keep_only(pids)
        mark = ",".join(f"{p}:{procs.start_time(p)}" for p in sorted(pids))
        patch = {"metadata": {
            "labels": {LABEL_OWNER: None, LABEL_OWNER_NS: None},
            "ownerReferences": None,
            "annotations": {ANN_MOUNT_MODE: MODE_DRAINING, ANN_DRAIN_PIDS: mark,
                            ANN_DRAIN_OWNER: f"{podu.ns_of(owner)}/{podu.name_of(owner)}",
                            ANN_OWNER_UID: None, ANN_IDEMPOTENCY: None, ANN_GROUP: None}}}
        kube = self.svc.ph.kube
        epoch = self.svc.ph.informer.epoch
        res = await asyncio.gather(*[kube.patch_pod(p.namespace, p.name, patch) for p in phs],
                                   return_exceptions=True)
        failed = []
        for ph, r in zip(phs, res):
            if isinstance(r, dict):
                self.svc.ph.informer.upsert(r, epoch)
                ph.mode = MODE_DRAINING
            else:
                _log.error("mark %s/%s draining: %s", ph.namespace, ph.name, r)
                failed.append(ph)
        marked = [ph for ph in phs if ph not in failed]
        if not marked:
            pinned.close()
            return failed
        for ph in marked:
            self.held[ph.uid] = (ph, pinned)
        self.svc.metrics.draining.set(len(self.held))
        self.svc.metrics.reconcile_actions.labels(action="drain_hold").inc(len(marked))
        log.kv(_log, 30, "GPU held until killed processes exit", pids=list(pids),
               placeholders=[p.name for p in marked])
        t = asyncio.ensure_future(self._wait(marked, pinned, list(pids)))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return failed

    async def _wait(self, phs: List[Placeholder], pinned: procs.Pinned, pids: List[int]) -> None:
        try:
            while pinned.fds:
                left = await pinned.wait_exit(pids, 3600.0)
                if not left:
                    break
            pinned.close()
            await self._release(phs)
        except asyncio.CancelledError:
            pinned.close()
            raise
        except Exception as e:  # noqa: BLE001 - the reconciler's sweep retries the release
            _log.error("drain release failed: %s", e)

    async def _release(self, phs: Sequence[Placeholder]) -> None:
        for ph in phs:
            self.held.pop(ph.uid, None)
        self.svc.metrics.draining.set(len(self.held))
        await self.svc.ph.release(list(phs), wait=False)
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
