"""Reconciler: repairs drift between the placeholder ledger and the node's actual device state.

The reference has no reconciliation: a container restart drops the mknod'd nodes
while the slave pod keeps the GPU, a worker crash mid-attach leaves rules behind, and the
cross-namespace ownerReference GC can delete slave pods under a live tenant (defects 4, 12).
Every ``reconcile_period_s`` (and on demand) this loop, per node:

1. deletes placeholders whose owner pod is gone or was replaced (UID mismatch) → ``owner_gone``;
2. deletes placeholders stuck Unschedulable/Failed that no in-flight attach is waiting on;
3. for every live owner, audits cgroup rules + ``/dev`` nodes against the ledger and re-applies
   missing ones (resume after a container restart) or revokes stale ones;
4. for every container the injection journal (node/journal.py) lists and no placeholder backs
   any more, revokes exactly the rules/nodes gpumounter recorded injecting there (orphans) — the
   "zero orphaned cgroup entries" invariant. Pods gpumounter never touched are never audited:
   their GPU nodes (a privileged pod's, the worker's own host ``/dev``, a device plugin's) are
   not gpumounter's state. Journal entries of containers that no longer run are dropped.
All repairs take the same per-pod lock as AddGPU/RemoveGPU.

The reference has no sweep at all; its only revocation path is RemoveGPU on the ledger-selected
GPUs of the named pod (reference: pkg/util/util.go:73-147, allocator.go:101-126).

Events are handled immediately instead of at the next sweep (:meth:`watch_events`): a
placeholder deleted by someone else (kubectl, eviction, preemption — its GPU goes back to the
scheduler, so the tenant's access is revoked within milliseconds, not a period later), a tenant
pod that is deleted or finished (its placeholders are released at once in ``pool`` namespace
mode, where no garbage collector does it) and a container restart (the hot-mounted GPUs go back
into the new container). A failed reaction is retried with backoff, and so is what a failed
attach/detach could not clean up (:meth:`follow_up`). A watch that relists missed events, so a
relist wakes the sweep; a sweep that hit errors runs again after a short backoff.
"""
from __future__ import annotations

import asyncio
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from gpumounter_amd.cluster.kube import NotFound
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.types import (ANN_ATTACH_ID, ANN_CANDIDATE, ANN_CONTAINER,
                                         ANN_INCARNATION, ANN_OWNER_UID)
from gpumounter_amd.utils import calls, log

_log = log.get("worker.reconciler")

Owner = tuple   # (name, namespace, uid) as a placeholder's labels and annotations name it


def _held(p: dict) -> tuple:
    """(namespace, name, uid, owner uid, attach id) of a placeholder as the cache holds it."""
    md = p["metadata"]
    ann = md.get("annotations") or {}
    return (md["namespace"], md["name"], md.get("uid", ""), ann.get(ANN_OWNER_UID) or "",
            ann.get(ANN_ATTACH_ID) or "")


def _owner_of(p: dict) -> Optional[Owner]:
    """The tenant a placeholder is booked for; None for warm-pool capacity (owned by the pool)
    and a force-removed GPU waiting for its killed processes (worker/drain.py)."""
    md = p["metadata"]
    ann = md.get("annotations") or {}
    if ann.get("gpumounter.amd.com/mount-mode") in ("standby", "draining"):
        return None
    return (ann.get("gpumounter.amd.com/owner-name", ""),
            (md.get("labels") or {}).get("gpumounter.amd.com/owner-namespace", ""),
            ann.get(ANN_OWNER_UID, ""))


@dataclass
class ReconcileReport:
    owner_gone: List[str] = field(default_factory=list)
    stuck: List[str] = field(default_factory=list)
    repaired: List[str] = field(default_factory=list)
    revoked: List[str] = field(default_factory=list)
    orphans: int = 0
    errors: List[str] = field(default_factory=list)
    claims_deleted: List[str] = field(default_factory=list)   # DRA mode: orphan claims
    drained: List[str] = field(default_factory=list)   # draining placeholders released
    # owners an attach/detach held locked: audited by a follow-up, swept again soon
    skipped: List[str] = field(default_factory=list)

    def to_dict(self) -> dict:
        return self.__dict__.copy()


class Reconciler:
    def __init__(self, service, period_s: float = 30.0, stuck_after_s: float = 120.0) -> None:
        self.svc = service
        self.period_s = period_s
        self.stuck_after_s = stuck_after_s
        self._task = None
        self.last: ReconcileReport = ReconcileReport()
        self._first_seen: Dict[str, float] = {}
        self._claim_seen: Dict[tuple, float] = {}
        self._kicked: set = set()
        self._timers: Dict[tuple, asyncio.TimerHandle] = {}   # retries of failed reactions
        self._bg: set = set()
        self.event_actions = 0
        self._stopping = False
        self._wake = asyncio.Event()
        self._last_sweep = 0.0
        self.woken = 0
        self.guard_period_s = float(getattr(getattr(service, "cfg", None),
                                            "device_guard_period_s", 0.0) or 0.0)
        self.guard_repairs = 0
        self._guard_task = None
        self._guard_timer = None
        self._guard_running: Optional[asyncio.Task] = None   # one pass at a time
        self._why: Dict[Tuple[str, str], str] = {}   # owner → cause of a pending revocation

    # ------------------------------------------------------------------------ events
    def watch_events(self) -> None:
        self.svc.ph.on_foreign_delete.append(self._on_foreign_delete)
        self.svc.node_pods.handlers.append(self._on_node_pod)
        self.svc.ph.informer.handlers.append(self._on_relist)

    def _on_relist(self, etype: str, _obj: dict) -> None:
        if etype == "RELIST":
            self.wake()

    def wake(self) -> None:
        """Sweep now rather than at the next period: a watch relisted (410 Gone, a dropped
        stream), so the events it missed — a container restart, a Pod or placeholder deleted —
        reached no reaction; the sweep finds what they would have triggered."""
        self._wake.set()

    def _on_foreign_delete(self, ph: dict) -> None:
        md = ph["metadata"]
        ann = md.get("annotations") or {}
        if ann.get("gpumounter.amd.com/mount-mode") in ("standby", "draining"):
            # pool capacity / a drain: no tenant has access to revoke. A standby preempted by a
            # higher-priority Pod (low pool_priority_class) is made up from what is free
            if ann.get("gpumounter.amd.com/mount-mode") == "standby":
                self._poke_pool()
            return
        ons = (md.get("labels") or {}).get("gpumounter.amd.com/owner-namespace", "")
        oname = ann.get("gpumounter.amd.com/owner-name", "")
        if oname:
            preempted = any(c.get("type") == "DisruptionTarget" and
                            c.get("reason") == "PreemptionByScheduler"
                            for c in (ph.get("status") or {}).get("conditions") or [])
            if preempted:
                # only a placeholder that ranks below a pending Pod can be a victim: the floor
                # PriorityClass is missing or was overridden (utils/doctor.py checks it)
                _log.error("placeholder %s/%s was PREEMPTED by the scheduler; revoking from "
                           "%s/%s", md.get("namespace"), md.get("name"), ons, oname)
                self.svc.metrics.reconcile_actions.labels(action="placeholder_preempted").inc()
                self._why[(ons, oname)] = "placeholder preempted by the scheduler"
            else:
                _log.warning("placeholder %s/%s deleted externally; revoking from %s/%s",
                             md.get("namespace"), md.get("name"), ons, oname)
            self._kick(("revoke", ons, oname))

    def _poke_pool(self) -> None:
        pool = getattr(self.svc, "pool", None)
        if pool is not None and pool.enabled:
            pool.poke()

    def _on_node_pod(self, etype: str, pod: dict) -> None:
        if etype == "RELIST":
            self.wake()
            return
        if etype == "DELETED" or podu.phase_of(pod) in ("Succeeded", "Failed"):
            pool = getattr(self.svc, "pool", None)
            if pool is not None and pool.enabled and pool.exhausted:
                self._poke_pool()           # capacity freed on this node: refill the pool
            if self.svc.ph.owned_by(pod, candidates=True):
                self._kick(("release", podu.ns_of(pod), podu.name_of(pod), podu.uid_of(pod)))
        elif etype == "MODIFIED" and self._restarted(pod):
            # a container of a Pod with hot-mounted GPUs was restarted: the new one starts with
            # the runtime's /dev and device rules, so the GPUs go back in now — not at the next
            # periodic sweep, by which time the restarted process has looked and found none
            self._kick(("reinject", podu.ns_of(pod), podu.name_of(pod)))
        elif etype == "MODIFIED" and self.guard_period_s > 0 and self._hot_cgroups(pod):
            # a Pod with hot-mounted GPUs changed (an in-place resize: runc update re-applies
            # the container's device rules): look again shortly, before the next guard tick
            self._guard_soon()

    # ------------------------------------------------------------------------ device guard
    def _hot_cgroups(self, pod: dict) -> List[str]:
        uid = podu.uid_of(pod)
        return [e.cgdir for e in self.svc.hm.journal.entries()
                if e.pod_uid == uid and e.rules and e.cgdir]

    def _guard_targets(self) -> List[tuple]:
        """(journal entry, cgroup dir) of every hot container with device rules."""
        return [(e, e.cgdir) for e in self.svc.hm.journal.entries() if e.rules and e.cgdir]

    @staticmethod
    def _fingerprints(fingerprint, dirs: List[str]) -> List[object]:
        """One syscall (BPF_PROG_QUERY) or one small read (devices.list) per cgroup, and
        whether the directory still exists: the part of a guard pass that touches the kernel,
        run off the event loop."""
        return [(fingerprint(d), os.path.isdir(d)) for d in dirs]

    def _guard_compare(self, targets: List[tuple], seen: List[object],
                       before: Dict[str, object]) -> List[tuple]:
        """The loop-side half of a pass: compare fingerprints taken at ``before`` (the expected
        state then) with what gpumounter expects now."""
        hm = self.svc.hm
        kicked = []
        live = set()
        for (e, d), (fp, exists) in zip(targets, seen):
            live.add(d)
            if d not in before:
                if d not in hm.expected:
                    hm.expected[d] = fp         # first sight (a restarted worker): baseline
                continue
            if hm.expected.get(d) is not before[d]:
                continue                        # gpumounter changed it meanwhile: next pass
            if fp != hm.expected[d] and exists:
                hm.expected[d] = fp             # kicked once; the repair records its own
                self.guard_repairs += 1
                _log.warning("device control of %s/%s changed outside gpumounter (%s); "
                             "re-checking its hot-mounted GPUs", e.namespace, e.pod, d)
                key = ("guard", e.namespace, e.pod)
                self._kick(key)
                kicked.append(key[1:])
        for d in [d for d in hm.expected if d not in live]:
            del hm.expected[d]
        return kicked

    def guard_once(self) -> List[tuple]:
        """Compare every hot container's device-control fingerprint with the one gpumounter left
        (node/hotmount.py ``expected``); a container whose state changed behind our back (the
        runtime re-attached its program, runc update, systemd, a devices.allow/deny write) has
        its pod reconciled now. Returns the (namespace, pod) pairs kicked. Synchronous: the
        periodic guard runs :meth:`guard_pass`, which fingerprints in a thread."""
        targets = self._guard_targets()
        fp = getattr(self.svc.hm.backend, "fingerprint", lambda d: None)
        before = dict(self.svc.hm.expected)
        return self._guard_compare(targets, self._fingerprints(fp, [d for _, d in targets]),
                                   before)

    async def guard_pass(self) -> List[tuple]:
        """:meth:`guard_once` with the kernel reads in the default executor: a node with many
        hot containers (CPX partitions: up to 64 per node) costs the RPC loop only the compare.
        A fingerprint taken while an attach or detach changed that cgroup is not compared (the
        expected state it was taken against is gone); the next pass looks again."""
        targets = self._guard_targets()
        if not targets:
            return self._guard_compare([], [], {})
        fp = getattr(self.svc.hm.backend, "fingerprint", lambda d: None)
        before = dict(self.svc.hm.expected)
        seen = await asyncio.to_thread(self._fingerprints, fp, [d for _, d in targets])
        return self._guard_compare(targets, seen, before)

    def _guard_soon(self, delay: float = 0.2) -> None:
        if self._guard_timer is None and not self._stopping:
            self._guard_timer = asyncio.get_running_loop().call_later(delay, self._guard_fire)

    def _guard_fire(self) -> None:
        self._guard_timer = None
        if self._guard_running is None or self._guard_running.done():
            self._guard_running = asyncio.ensure_future(self._guard_safe())

    async def _guard_safe(self) -> None:
        try:
            await self.guard_pass()
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - the next tick or the sweep retries
            _log.warning("device guard: %s", e)

    async def _guard_loop(self) -> None:
        while True:
            await asyncio.sleep(self.guard_period_s)
            self._guard_fire()

    def _restarted(self, pod: dict) -> bool:
        """A running container of a Pod that holds hot-mounted GPUs has no injection record:
        it started after the attach (a restart), or its record is lost."""
        phs = self.svc.ph.owned_by(pod)
        if not phs or podu.phase_of(pod) != "Running":
            return False
        wanted = {(p["metadata"].get("annotations") or {}).get(ANN_CONTAINER, "") for p in phs}
        journal = self.svc.hm.journal
        return any(r.running and not r.privileged and ("" in wanted or r.name in wanted)
                   and journal.get(r.id) is None for r in podu.running_containers(pod))

    # a failed reaction (apiserver error, a kernel call refused) is retried after these delays
    # before it is left to the periodic sweep, which may be 30 s away
    RETRY_DELAYS = (0.1, 0.5, 2.0, 5.0)

    def follow_up(self, ns: str, name: str, drop=()) -> None:
        """Finish what a failed operation on ``ns/name`` left: release the placeholders in
        ``drop`` that still exist, then reconcile the Pod to its ledger. Retried with backoff
        (the kubelet restarting, the apiserver failing) like an event reaction."""
        self._kick(("followup", ns, name,
                    tuple(sorted((p.namespace, p.name, p.uid, p.owner_uid, p.attach_id)
                                 for p in drop))))

    def _kick(self, key: tuple, attempt: int = 0) -> None:
        if key in self._kicked or self._stopping:
            return
        self._kicked.add(key)
        t = asyncio.ensure_future(self._react(key, attempt))
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    def _retry(self, key: tuple, attempt: int) -> None:
        if attempt > len(self.RETRY_DELAYS) or key in self._timers or self._stopping:
            return
        loop = asyncio.get_running_loop()
        self._timers[key] = loop.call_later(self.RETRY_DELAYS[attempt - 1], self._fire, key,
                                            attempt)

    def _fire(self, key: tuple, attempt: int) -> None:
        self._timers.pop(key, None)
        self._kick(key, attempt)

    async def _react(self, key: tuple, attempt: int = 0) -> None:
        calls.mark_background()
        svc = self.svc
        await asyncio.sleep(0)  # coalesce a burst of events for one owner
        self._kicked.discard(key)
        ns, name = key[1], key[2]
        try:
            async with svc.pod_lock(ns, name):
                if key[0] == "release":
                    stub = {"metadata": {"namespace": ns, "name": name, "uid": key[3]}}
                    phs = svc.ph.owned_by(stub, candidates=True)
                    if phs:   # back to the warm pool when one is configured
                        await svc._release([svc.ph.cached(p) or svc.ph.from_pod(p, {})
                                            for p in phs])
                        svc.metrics.orphans.labels(kind="owner_gone").inc(len(phs))
                else:
                    owner = svc.node_pods.get(ns, name)
                    if key[0] == "followup":
                        if key[3]:
                            await self._drop(sorted(key[3]))
                        # candidates of a pick are never an owner's; under the pod's lock no
                        # pick is running, so any left belong to a failed one. The cache may
                        # predate the pick's confirm (a relist), so each goes only if the
                        # apiserver still shows it a candidate
                        cands = [] if owner is None else [
                            p for p in svc.ph.owned_by(owner, candidates=True)
                            if ANN_CANDIDATE in (p["metadata"].get("annotations") or {})]
                        if cands:
                            await self._drop(sorted({_held(p) for p in cands} - set(key[3])),
                                             candidates_only=True)
                    if owner is None or podu.phase_of(owner) != "Running":
                        return
                    fixed = await svc.reconcile_pod(owner)
                    gone = sorted({i.path for i in fixed if i.kind.startswith("stale")})
                    back = sorted({i.path for i in fixed if i.kind.startswith("missing")})
                    why = self._why.pop((ns, name), "placeholder deleted outside gpumounter")
                    if gone:
                        svc.notify.event(owner, "GPURevoked",
                                         f"{why}; access revoked: {', '.join(gone)}",
                                         warning=True)
                    if back and key[0] == "reinject":
                        svc.notify.event(owner, "GPUReinjected",
                                         f"container restarted; hot-mounted devices restored: "
                                         f"{', '.join(back)}")
                    elif back and key[0] == "guard":
                        svc.notify.event(owner, "GPUReinjected",
                                         f"device rules were replaced outside gpumounter "
                                         f"(runtime, runc update or systemd); hot-mounted "
                                         f"access restored: {', '.join(back)}", warning=True)
                self.event_actions += 1
                svc.metrics.reconcile_actions.labels(action=f"event_{key[0]}").inc()
        except asyncio.CancelledError:
            if self._stopping:
                raise
            # not ours: something this reaction awaited was cancelled under it (see _loop)
            _log.error("event-driven reconcile %s was cancelled (attempt %d)", key, attempt + 1)
            svc.metrics.reconcile_actions.labels(action="event_retry").inc()
            self._retry(key, attempt + 1)
        except Exception as e:  # noqa: BLE001 - retried, then the periodic sweep
            _log.error("event-driven reconcile %s failed (attempt %d): %s", key, attempt + 1, e)
            svc.metrics.reconcile_actions.labels(action="event_retry").inc()
            self._retry(key, attempt + 1)

    async def _drop(self, phs, candidates_only: bool = False) -> None:
        """Release the placeholders of a failed attach that still exist (same UID), each only
        while it has the holder the attach left it with: one that went back to the warm pool
        and was claimed since (by another Pod, or by a later attach of this one) is not the
        failed attach's to release (cluster/placeholder.py ``_delete``, pool ``give_back``).
        ``candidates_only``: found as unconfirmed candidates in the cache, each deleted only
        while the apiserver still shows it one."""
        svc = self.svc
        left = []
        for ns, name, uid, owner_uid, attach_id in phs:
            p = svc.ph.informer.cache.get((ns, name))
            if p is not None and (not uid or p["metadata"].get("uid") == uid) and \
                    not p["metadata"].get("deletionTimestamp"):
                ph = svc.ph.cached(p) or svc.ph.from_pod(p, {})
                ph.owner_uid, ph.attach_id = owner_uid, attach_id
                left.append(ph)
        if left:
            if candidates_only:
                await svc.ph.release(left, candidates_only=True)
            else:
                await svc._release(left)
            svc.metrics.reconcile_actions.labels(action="followup_release").inc(len(left))
        for _, _, uid, _, _ in phs:
            svc.abandoned.pop(uid, None)

    async def start(self) -> None:
        self._task = asyncio.ensure_future(self._loop())
        self.start_guard()

    def start_guard(self) -> None:
        """The device guard runs whether or not the periodic sweep does."""
        if self.guard_period_s > 0 and self._guard_task is None:
            self._guard_task = asyncio.ensure_future(self._guard_loop())

    async def stop(self) -> None:
        self._stopping = True
        if self._guard_task is not None:
            self._guard_task.cancel()
        if self._guard_timer is not None:
            self._guard_timer.cancel()
        if self._guard_running is not None:
            self._guard_running.cancel()
        for h in list(self._timers.values()):
            h.cancel()
        self._timers.clear()
        for t in list(self._bg):
            t.cancel()
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass

    # a sweep that could not finish everything (the kubelet restarting, the apiserver failing, a
    # kernel call refused) runs again after these delays rather than a whole period later
    SWEEP_RETRY_DELAYS = (0.5, 2.0, 5.0, 10.0)
    # a sweep that skipped an owner an operation held sweeps again this soon (found by chaos:
    # a restarted worker's first sweep skipped the owner its lease expiry held, and that
    # owner's placeholders from the dead worker's last attach stayed unbound for a period)
    SKIPPED_RESWEEP_S = 2.0
    # woken sweeps (relists) run at most this often: a flapping watch must not turn into a
    # PodResources List per relist
    WAKE_MIN_INTERVAL_S = 1.0

    async def _loop(self) -> None:
        calls.mark_background()
        # the first sweep runs at once: whatever changed while no worker was running (a
        # container restarted, a Pod deleted, an attach cut off by the previous worker's death)
        # sent its events to nobody, and the next periodic sweep may be 30 s away
        delay, failures = 0.0, 0
        loop = asyncio.get_running_loop()
        # not `while True`: on Python 3.10 asyncio.wait_for can swallow the stop's cancellation
        # when the wake-up lands at the same moment; the flag ends the loop regardless
        while not self._stopping:
            if delay:
                try:
                    await asyncio.wait_for(self._wake.wait(), delay)
                    self.woken += 1
                    await asyncio.sleep(max(0.0, self._last_sweep + self.WAKE_MIN_INTERVAL_S
                                            - loop.time()))
                except asyncio.TimeoutError:
                    pass
            self._wake.clear()
            self._last_sweep = loop.time()
            skipped = False
            try:
                rep = await self.run_once()
                ok, skipped = not rep.errors, bool(rep.skipped)
            except asyncio.CancelledError:
                if self._stopping:
                    raise
                # a CancelledError that stop() did not cause came from something the sweep
                # awaited (a cancelled inner future): a failed sweep, not the end of the loop
                _log.error("reconcile sweep was cancelled from within; retrying")
                ok = False
            except Exception as e:  # noqa: BLE001
                _log.exception("reconcile failed: %s", e)
                ok = False
            if ok:
                delay, failures = self.period_s, 0
                if skipped:
                    delay = min(self.period_s, self.SKIPPED_RESWEEP_S)
            else:
                delay = min(self.period_s, self.SWEEP_RETRY_DELAYS[
                    min(failures, len(self.SWEEP_RETRY_DELAYS) - 1)])
                failures += 1

    async def _sweep_claims(self) -> List[str]:
        """DRA mode: our ResourceClaims whose placeholder Pod does not exist (a worker that died
        between creating the claim and the Pod, a Pod deleted by someone else) and that no Pod
        holds. They hold no device, so this is cleanup; a claim gets ``stuck_after_s`` to be
        joined by its Pod first."""
        svc = self.svc
        ns = "" if svc.cfg.placeholder_namespace_mode == "tenant" else svc.cfg.pool_namespace
        claims = await svc.kube.list_claims(ns, svc.ph.selector_for_node(svc.ph.node))
        now = time.monotonic()
        out, seen = [], set()
        for c in claims:
            md = c["metadata"]
            key = (md.get("namespace", ""), md.get("name", ""))
            seen.add(key)
            if svc.ph.informer.cache.get(key) is not None or \
                    (c.get("status") or {}).get("reservedFor"):
                self._claim_seen.pop(key, None)
                continue
            if now - self._claim_seen.setdefault(key, now) < self.stuck_after_s:
                continue
            try:
                await svc.kube.delete_claim(*key)
            except NotFound:
                pass
            self._claim_seen.pop(key, None)
            out.append(f"{key[0]}/{key[1]}")
        for key in [k for k in self._claim_seen if k not in seen]:
            del self._claim_seen[key]
        if out:
            svc.metrics.reconcile_actions.labels(action="claim_delete").inc(len(out))
        return out

    async def _owned_now(self, owner: Owner) -> Optional[List[dict]]:
        """``owner``'s placeholders as the informer holds them now, once no write-through of
        ours is waiting to be re-read after a relist (see ``WorkerService.pod_state``); None if
        the view did not settle in time."""
        inf = self.svc.ph.informer
        if not getattr(inf, "settled", True):
            try:
                await inf.wait_for(lambda: inf.settled,
                                   getattr(self.svc, "SETTLE_WAIT_S", 2.0))
            except asyncio.TimeoutError:
                return None
        return [p for p in self.svc.ph.live() if _owner_of(p) == owner]

    async def run_once(self) -> ReconcileReport:
        svc = self.svc
        rep = ReconcileReport()
        try:
            await svc.lease.sweep()            # leases that expired while nobody watched
        except Exception as e:  # noqa: BLE001
            rep.errors.append(f"lease sweep: {e}")
        svc.hm.backend.prune()
        m = svc.metrics
        # One authoritative PodResources read per sweep. It cross-checks the device-manager
        # checkpoint, and while that stays trusted every owner is audited from it (re-read
        # under the owner's lock, no RPC). That is O(1) kubelet calls per sweep instead of one
        # per owner.
        led: Optional[Dict[tuple, List[str]]] = None
        try:
            led = await svc.read_ledger(authoritative=True)
        except Exception as e:  # noqa: BLE001
            rep.errors.append(f"ledger: {e}")
        if not svc.adopted:
            try:
                await svc.adopt_existing()
            except Exception as e:  # noqa: BLE001
                rep.errors.append(f"journal adoption: {e}")
        ck = svc.ph.checkpoint
        from_ckpt = ck is not None and ck.trusted and ck.snapshot() is not None
        placeholders = svc.ph.live()
        by_owner: Dict[Owner, List[dict]] = {}
        for p in placeholders:
            owner = _owner_of(p)
            if owner is not None:
                by_owner.setdefault(owner, []).append(p)
        now = time.monotonic()
        async def fresh(ns: str, name: str):
            try:
                return await svc.kube.get_pod(ns, name)
            except NotFound:
                return None

        def gone(p, uid: str) -> bool:
            return p is None or podu.uid_of(p) != uid or podu.phase_of(p) in ("Succeeded",
                                                                              "Failed")

        async def collect(ons: str, oname: str, phs: List[dict]) -> None:
            # a force-removed GPU whose draining mark is pending stays booked until its killed
            # processes are gone (worker/drain.py), owner or not
            phs = [p for p in phs if p["metadata"].get("uid") not in svc.drain.unmarked]
            for p in phs:
                rep.owner_gone.append(p["metadata"]["name"])
                m.orphans.labels(kind="owner_gone").inc()
            await svc.ph.release([svc.ph.from_pod(p, {}) for p in phs])

        for key in by_owner:
            oname, ons, ouid = key
            # the node informer already holds every pod of this node; the apiserver is only
            # asked to confirm an owner the cache shows gone/replaced, or whose repair failed
            owner = svc.node_pods.get(ons, oname)
            if gone(owner, ouid):
                owner = await fresh(ons, oname)
            lock = svc.pod_lock(ons, oname)
            if gone(owner, ouid):
                async with lock:
                    phs = await self._owned_now(key)
                    if phs is None:
                        rep.errors.append(f"{ons}/{oname}: placeholder view not settled")
                    elif phs:
                        await collect(ons, oname, phs)
                continue
            if lock.locked():
                # an attach/detach is in flight for this owner: audit it right after, not a
                # period later (the events this sweep stands in for, a container restart
                # missed by a relist, say, will not come again); its placeholders (a dead
                # worker's unadmitted ones, a failed pick's) wait for the next sweep, which
                # comes SKIPPED_RESWEEP_S later instead of a period
                self.follow_up(ons, oname)
                rep.skipped.append(f"{ons}/{oname}")
                continue
            async with lock:
                # the snapshot above is older than this lock: an attach that held it meanwhile
                # confirmed its pick (candidates no more) or added or released placeholders.
                # Judged from that snapshot, a just-confirmed pick reads as abandoned and is
                # released under the Pod it was mounted in
                phs = await self._owned_now(key)
                if phs is None:
                    rep.errors.append(f"{ons}/{oname}: placeholder view not settled")
                    continue
                # candidates of a trim/correction pick whose attach is not running (its worker
                # died mid-pick): never the owner's, never mounted — give the GPUs back
                # and placeholders of failed attaches whose release the follow-up gave up on
                marked = [p for p in phs
                          if ANN_CANDIDATE in (p["metadata"].get("annotations") or {})
                          and not svc.is_abandoned(p)]
                cands = marked + [p for p in phs if svc.is_abandoned(p)]
                if cands:
                    rep.stuck += [p["metadata"]["name"] for p in cands]
                    # a candidate mark in the cache is only gone once the confirm's write is
                    # re-read: the apiserver decides (cluster/placeholder.py _delete)
                    await svc.ph.release([svc.ph.from_pod(p, {}) for p in marked],
                                         candidates_only=True)
                    await svc.ph.release([svc.ph.from_pod(p, {}) for p in cands
                                          if p not in marked])
                    for p in cands:
                        svc.abandoned.pop(p["metadata"].get("uid", ""), None)
                    phs = [p for p in phs if p not in cands]
                    m.reconcile_actions.labels(action="candidate_release").inc(len(cands))
                # stuck placeholders (never admitted). One that an earlier worker process
                # created and that the kubelet has not allocated devices to belongs to an
                # attach that died with that worker: nothing waits for it, and if the scheduler
                # admitted it later the reconciler would mount GPUs nobody asks for any more —
                # released at once. (An admitted one may be a finished attach whose reply was
                # sent: it stays, and is audited like any other.)
                stuck = []
                for p in phs:
                    name = p["metadata"]["name"]
                    ann = p["metadata"].get("annotations") or {}
                    if led is not None and podu.phase_of(p) == "Pending" and \
                            not led.get((p["metadata"]["namespace"], name)) and \
                            ann.get(ANN_INCARNATION) != svc.ph.incarnation:
                        stuck.append(p)
                        m.reconcile_actions.labels(action="dead_attach_release").inc()
                    elif podu.phase_of(p) == "Failed" and led is not None and \
                            not led.get((p["metadata"]["namespace"], name)):
                        # refused at admission (OutOf<resource>: a directly bound placeholder
                        # on a full node) and no attach of this owner is running (its lock is
                        # held): terminal, it holds no device
                        stuck.append(p)
                        m.reconcile_actions.labels(action="failed_release").inc()
                    elif podu.is_unschedulable(p) or podu.phase_of(p) == "Failed":
                        first = self._first_seen.setdefault(name, now)
                        if now - first >= self.stuck_after_s:
                            stuck.append(p)
                if stuck:
                    rep.stuck += [p["metadata"]["name"] for p in stuck]
                    await svc.ph.release([svc.ph.from_pod(p, {}) for p in stuck])
                if podu.phase_of(owner) != "Running":
                    continue
                try:
                    fixed = await svc.reconcile_pod(owner, authoritative=not from_ckpt)
                except Exception as e:  # noqa: BLE001
                    if gone(await fresh(ons, oname), ouid):   # the cache lagged a delete
                        await collect(ons, oname, phs)
                    else:
                        rep.errors.append(f"{ons}/{oname}: {e}")
                    continue
                if fixed:
                    rep.orphans += sum(1 for i in fixed if i.kind.startswith("stale"))
                    rep.repaired.append(f"{ons}/{oname}")
                    m.reconcile_actions.labels(action="repair").inc()
        # journaled hot-mount state that no placeholder backs any more must not stay behind
        owners = {(o[1], o[0], o[2]) for o in by_owner}
        journal = svc.hm.journal
        for ent in journal.entries():
            pod = svc.node_pods.get(ent.namespace, ent.pod)
            alive = pod is not None and podu.uid_of(pod) == ent.pod_uid and \
                podu.phase_of(pod) == "Running" and any(
                    r.id == ent.container_id and r.running
                    for r in podu.running_containers(pod))
            if not alive:
                # container gone: its cgroup and mount namespace (and our state) went with it.
                # Confirmed with the apiserver first, so a lagging cache never loses a record
                pod = await fresh(ent.namespace, ent.pod)
                if pod is None or podu.uid_of(pod) != ent.pod_uid or not any(
                        r.id == ent.container_id and r.running
                        for r in podu.running_containers(pod)):
                    journal.drop(ent.container_id)
                    continue
            if (ent.namespace, ent.pod, ent.pod_uid) in owners:
                continue            # audited against its placeholders above
            key = (ent.namespace, ent.pod)
            lock = svc.pod_lock(*key)
            if lock.locked():
                self.follow_up(*key)        # as above: once the operation in flight is done
                rep.skipped.append("/".join(key))
                continue
            async with lock:
                if svc.ph.owned_by(pod):
                    continue        # an attach completed meanwhile
                try:
                    revoked = svc.hm.revoke_journaled(pod, ent.container_id)
                except Exception as e:  # noqa: BLE001
                    rep.errors.append(f"revoke {key}: {e}")
                    continue
                if revoked:
                    rep.orphans += len(revoked)
                    m.orphans.labels(kind="stale_state").inc(len(revoked))
                    name = f"{key[0]}/{key[1]}"
                    if name not in rep.revoked:
                        rep.revoked.append(name)
                    m.reconcile_actions.labels(action="revoke").inc()
        try:
            rep.drained = await svc.drain.sweep()
        except Exception as e:  # noqa: BLE001
            rep.errors.append(f"drain sweep: {e}")
        for name in list(self._first_seen):
            if not any(p["metadata"]["name"] == name for p in placeholders):
                del self._first_seen[name]
        sweep = getattr(svc.hm.backend, "sweep_pins", None)
        if sweep is not None:
            try:
                # a walk of the whole cgroup tree: off the event loop, attaches keep flowing
                gone = await asyncio.to_thread(sweep, svc.hm.resolver.root)
            except Exception as e:  # noqa: BLE001
                rep.errors.append(f"bpf pin sweep: {e}")
            else:
                if gone:
                    m.reconcile_actions.labels(action="unpin").inc(len(gone))
        if svc.ph.dra:
            try:
                rep.claims_deleted = await self._sweep_claims()
            except Exception as e:  # noqa: BLE001
                rep.errors.append(f"resourceclaim sweep: {e}")
        self.last = rep
        if rep.owner_gone or rep.stuck or rep.repaired or rep.revoked or rep.errors or \
                rep.claims_deleted or rep.drained:
            log.kv(_log, 20, "reconciled", **rep.to_dict())
        return rep
