"""GPU leases: hot-mounted GPUs that give themselves back.

``GET /addgpu/...?lease=3600`` attaches GPUs for an hour. The expiry time is stored on the
placeholder pods (annotation ``gpumounter.amd.com/lease-expires``, Unix seconds), so it survives
worker restarts: a timer detaches on time while the worker runs, and the reconciler's sweep
catches any lease that expired while it did not. Expiry is an ordinary RemoveGPU with the
requester ``lease-expiry``. A GPU still in use is kept (``GPULeaseExpired`` warning Event,
retried every ``lease_retry_s``) unless ``lease_force`` is set, in which case its processes get
the same SIGTERM→SIGKILL treatment as ``force=1``. The reference has no notion of time-bounded
mounts; its slave pods live until someone removes them (reference: pkg/server/gpu-mount/
server.go:101-179).
"""
from __future__ import annotations

import asyncio
import time
from typing import Dict, List, Optional, Tuple

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.types import (ANN_ATTACH_ID, ANN_GROUP, ANN_LEASE,
                                         ANN_OWNER_UID, LABEL_OWNER_NS, MountType)
from gpumounter_amd.node.ledger import LedgerError
from gpumounter_amd.utils import calls, log

_log = log.get("worker.lease")
__all__ = ["ANN_LEASE", "LeaseKeeper", "expires_of"]


def _holder(ph: dict) -> Tuple[str, str]:
    """The attach a placeholder serves now: (owner pod uid, attach id)."""
    ann = ph["metadata"].get("annotations") or {}
    return ann.get(ANN_OWNER_UID) or "", ann.get(ANN_ATTACH_ID) or ""


def expires_of(ph: dict) -> Optional[float]:
    v = (ph["metadata"].get("annotations") or {}).get(ANN_LEASE)
    try:
        return float(v) if v else None
    except ValueError:
        return None


class LeaseKeeper:
    def __init__(self, service) -> None:
        self.svc = service
        # placeholder uid → (timer, the expiry it was armed for)
        self._timers: Dict[str, Tuple[asyncio.TimerHandle, float]] = {}
        # placeholder uid → not before: a lease whose GPUs were busy at expiry (lease_force off)
        # is retried every lease_retry_s. Per placeholder: a later lease of the same owner is
        # not held back by it
        self._retry_after: Dict[str, float] = {}
        self._retry_timers: Dict[Tuple[str, str], asyncio.TimerHandle] = {}
        self._errors: Dict[Tuple[str, str], int] = {}          # owner → failed expiries in a row
        self._tasks: set = set()                               # running expiries
        self._locks: Dict[Tuple[str, str], asyncio.Lock] = {}  # owner → its expiries in turn
        # placeholder uid → (expiry this worker granted, the holding attach: owner pod uid,
        # attach id): the informer learns the annotation only from the watch echo of our PATCH,
        # which can lag (a dropped stream, a relist). A warm-pool placeholder changes hands, also
        # back to the same Pod by a later attach, so a grant holds only for the attach it was
        # made for (see _holder)
        self._granted: Dict[str, Tuple[float, Tuple[str, str]]] = {}
        # placeholder uid → times its expired lease was found not admitted yet (backoff)
        self._waits: Dict[str, int] = {}
        self._stopped = False
        self.expired = 0

    # ------------------------------------------------------------------------ grant
    async def grant(self, pod: dict, placeholders, lease_s: float) -> float:
        """Stamp the expiry on placeholders booked without it and arm a timer; returns the
        expiry. Attaches write their lease with the booking (:meth:`booked`); this is for the
        replay of an attach an older worker (one PATCH after the mount) left unleased."""
        expires = time.time() + lease_s
        patch = {"metadata": {"annotations": {ANN_LEASE: f"{expires:.3f}"}}}
        informer = self.svc.ph.informer
        epoch = informer.epoch
        res = await asyncio.gather(*[self.svc.kube.patch_pod(p.namespace, p.name, patch)
                                     for p in placeholders])
        for p, r in zip(placeholders, res):
            if isinstance(r, dict):
                informer.upsert(r, epoch)    # visible to expire_owner before the watch echo
                if p.uid:
                    self._granted[p.uid] = (expires, _holder(r))
            self._arm(p.uid, podu.ns_of(pod), podu.name_of(pod), expires)
        return expires

    def booked(self, pod: dict, placeholders, expires: float) -> None:
        """An attach whose placeholders were created or claimed with the lease annotation
        (cluster/placeholder.py ``build``, cluster/pool.py ``claim``): remember the grant and arm
        the timers; nothing is written."""
        for p in placeholders:
            if p.uid:
                self._granted[p.uid] = (expires, (p.owner_uid, p.attach_id))
            self._arm(p.uid, podu.ns_of(pod), podu.name_of(pod), expires)

    def granted(self, raw: dict) -> Optional[float]:
        """The expiry this worker granted to placeholder ``raw`` for the attach that holds it
        now (None: none, or granted to an earlier holder of a warm-pool placeholder)."""
        g = self._granted.get(raw["metadata"].get("uid", ""))
        return g[0] if g is not None and g[1] == _holder(raw) else None

    def _arm(self, uid: str, ns: str, name: str, expires: float) -> None:
        """A timer for the lease of placeholder ``uid`` (one per placeholder; re-arming an
        armed one for a different expiry replaces it)."""
        if not uid or self._stopped:
            return
        old = self._timers.get(uid)
        if old is not None:
            if abs(old[1] - expires) < 1e-3:
                return
            old[0].cancel()
        loop = asyncio.get_running_loop()
        self._timers[uid] = (loop.call_later(max(0.0, expires - time.time()), self._fired,
                                             uid, ns, name), expires)

    def _fired(self, uid: str, ns: str, name: str) -> None:
        self._timers.pop(uid, None)          # spent: a later _arm must create a new one
        self._spawn(ns, name)

    def _spawn(self, ns: str, name: str) -> None:
        """Timer callback: run one expiry as a tracked task (cancelled by stop())."""
        if self._stopped:
            return
        task = asyncio.ensure_future(self._expire_or_retry(ns, name))
        self._tasks.add(task)
        task.add_done_callback(self._tasks.discard)

    # an expiry that failed (the apiserver or the kubelet erring, a node operation refused) is
    # retried after these delays, then every lease_retry_s: not left to the periodic sweep.
    # Doubling from 0.1 s: three transient failures in a row end the lease 0.7 s late, not
    # 2.6 s (chaos hpl312: three injected unmount faults, then a 2 s wait)
    ERROR_RETRY_S = (0.1, 0.2, 0.4, 0.8, 1.6)

    async def _expire_or_retry(self, ns: str, name: str) -> None:
        calls.mark_background()
        # one expiry per owner at a time: the timers of an attach's placeholders fire together,
        # and a second expiry racing the first would find its GPUs gone (GPUNotFound)
        lock = self._locks.setdefault((ns, name), asyncio.Lock())
        try:
            async with lock:
                await self.expire_owner(ns, name)
            self._errors.pop((ns, name), None)
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - retried below
            n = self._errors.get((ns, name), 0)
            self._errors[(ns, name)] = n + 1
            delay = self.ERROR_RETRY_S[n] if n < len(self.ERROR_RETRY_S) else \
                self.svc.cfg.lease_retry_s
            fast = len(self.ERROR_RETRY_S)
            _log.log(40 if n <= fast else 30,
                     "lease expiry of %s/%s failed (attempt %d, retry in %g s): %s",
                     ns, name, n + 1, delay, e)
            if n == fast:
                # the quick retries did not get through: tell the Pod's owner once, then keep
                # trying at the slow period (the ledger is re-read every time)
                pod = self.svc.node_pods.get(ns, name) if hasattr(self.svc, "node_pods") \
                    else None
                if pod is not None:
                    self.svc.notify.event(
                        pod, "GPULeaseExpired",
                        f"lease over, but the GPUs could not be detached: {e}; retrying "
                        f"every {self.svc.cfg.lease_retry_s:g} s", warning=True)
            if not self._stopped:
                old = self._retry_timers.pop((ns, name), None)
                if old is not None:
                    old.cancel()
                self._retry_timers[(ns, name)] = asyncio.get_running_loop().call_later(
                    delay, self._spawn, ns, name)

    async def stop(self, grace_s: float = 5.0) -> None:
        """Worker shutdown: no timer fires afterwards, and an expiry already detaching is
        allowed ``grace_s`` to finish (it is an ordinary RemoveGPU) before it is cancelled, so
        nothing runs against the closed clients. The next worker's start-up sweep picks the
        remaining leases up from the placeholder annotations."""
        self._stopped = True
        for t in [h for h, _ in self._timers.values()] + list(self._retry_timers.values()):
            t.cancel()
        self._timers.clear()
        self._retry_timers.clear()
        if self._tasks:
            _, late = await asyncio.wait(list(self._tasks), timeout=grace_s)
            for task in late:
                task.cancel()

    # ------------------------------------------------------------------------ expiry
    async def sweep(self, expire_due: bool = True) -> int:
        """Expire every lease that is due (placeholder annotations: survives worker restarts)
        and re-arm timers for the rest. Returns how many owners were due. A worker re-arms
        (``expire_due=False``) before it serves its first request, and expires what is due
        once it is up. A failed expiry is retried like a timer's (0.1 s doubling to 1.6 s, then
        ``lease_retry_s``)."""
        now = time.time()
        due: Dict[Tuple[str, str], List[dict]] = {}
        live = self.svc.ph.live()
        owners = {p["metadata"].get("uid"): _holder(p) for p in live}
        for uid in [u for u, (_, o) in self._granted.items()
                    if u not in owners or owners[u] != o]:
            del self._granted[uid]          # released some other way (RemoveGPU, owner gone,
            #                                 back in the warm pool)
        for uid in [u for u in self._retry_after if u not in owners]:
            del self._retry_after[uid]
        for uid in [u for u in self._waits if u not in owners]:
            del self._waits[uid]
        for key in [k for k, lk in self._locks.items() if not lk.locked()]:
            del self._locks[key]
        for p in live:
            exp = expires_of(p)
            if exp is None:
                continue
            md = p["metadata"]
            ns = (md.get("labels") or {}).get(LABEL_OWNER_NS, "")
            name = (md.get("annotations") or {}).get("gpumounter.amd.com/owner-name", "")
            if not (ns and name):
                continue
            if exp <= now:
                due.setdefault((ns, name), []).append(p)
            else:
                self._arm(md.get("uid", ""), ns, name, exp)
        if expire_due:
            for ns, name in due:
                await self._expire_or_retry(ns, name)
        return len(due)

    async def expire_owner(self, ns: str, name: str) -> None:
        svc = self.svc
        pod = await svc.get_pod(ns, name, fresh=True)
        if pod is None:
            return                          # the owner-gone GC releases its placeholders
        now = time.time()
        st = await svc.pod_state(pod, fresh=True)
        raws = {p["metadata"]["name"]: p for p in svc.ph.owned_by(pod)}
        if st.mount_type == MountType.UNKNOWN:
            # the ledger is unreadable right now (kubelet restarting, a claim not in the watch
            # cache yet): fail, so the expiry is retried shortly — returning would drop it
            raise LedgerError(f"lease expiry of {ns}/{name}: ledger unavailable")
        known = {ph.name for ph in st.placeholders}
        for pname, raw in raws.items():
            exp = expires_of(raw)
            if pname not in known and exp is not None and exp <= now + 0.001:
                # a leased placeholder of this owner the ledger view does not resolve yet
                raise LedgerError(f"lease expiry of {ns}/{name}: placeholder {pname} is not "
                                  f"in the ledger yet")
        uuids, due = [], []
        for ph in st.placeholders:
            raw = raws.get(ph.name)
            exp = expires_of(raw) if raw is not None else None
            if exp is None and raw is not None:
                exp = self.granted(raw)
            if exp is None:
                continue
            if exp <= now + 0.001:
                if now + 0.05 < self._retry_after.get(ph.uid, 0):
                    continue                # busy at its last expiry: its retry timer runs
                if not st.by_placeholder.get((ph.namespace, ph.name)):
                    # not admitted yet (a dead worker's attach, a scheduler slower than the
                    # lease): its GPU comes with admission, and the reconciler mounts it. Looked
                    # at again shortly (backing off to lease_retry_s) until it holds GPUs or is
                    # gone, not left to the next periodic sweep
                    n = self._waits.get(ph.uid, 0)
                    self._waits[ph.uid] = min(n + 1, 16)
                    self._arm(ph.uid, ns, name,
                              now + min(0.1 * 2 ** n, self.svc.cfg.lease_retry_s))
                    continue
                self._waits.pop(ph.uid, None)
                due.append(ph.uid)
                uuids += [g.uuid for g in st.by_placeholder[(ph.namespace, ph.name)]]
                t = self._timers.pop(ph.uid, None)
                if t is not None:
                    t[0].cancel()
            else:
                # not due yet (a timer of an earlier lease of this owner, or one that fired a
                # hair early): keep a timer for this one, it must not be lost
                self._arm(ph.uid, ns, name, exp)
        if not uuids:
            return
        # an entire mount comes and goes whole: a lease on part of its group (the grant was
        # cut off by a worker restart) ends the whole group, or the removal is refused as partial
        def group(ph) -> str:
            raw = raws.get(ph.name)
            return ((raw or {}).get("metadata", {}).get("annotations") or {}).get(ANN_GROUP) or ""
        groups = {group(ph) for ph in st.placeholders if ph.uid in due} - {""}
        for ph in st.placeholders:
            if ph.uid not in due and group(ph) in groups:
                due.append(ph.uid)
                uuids += [g.uuid for g in st.by_placeholder[(ph.namespace, ph.name)]]
        force = bool(svc.cfg.lease_force)
        resp = await svc.remove_gpu(api.RemoveGPURequest(
            pod_name=name, namespace=ns, uuids=uuids, force=force, requested_by="lease-expiry"))
        if resp.remove_gpu_result == api.REMOVE_SUCCESS:
            for uid in due:
                self._granted.pop(uid, None)
                self._retry_after.pop(uid, None)
            self.expired += 1
            svc.notify.event(pod, "GPULeaseExpired",
                             f"lease over: {len(uuids)} GPU(s) detached"
                             + (f", processes {list(resp.killed_pids)} signalled"
                                if resp.killed_pids else ""))
            log.kv(_log, 20, "lease expired", pod=f"{ns}/{name}", gpus=len(uuids))
            return
        if resp.remove_gpu_result != api.REMOVE_BUSY:
            # some of them went meanwhile (a client's RemoveGPU, the Pod deleted): read the
            # ledger again shortly (the error path's 0.1 … 1.6 s retries) for what is left
            raise LedgerError(
                f"lease expiry of {ns}/{name}: "
                f"{api.RemoveGPUResponse.RemoveGPUResult.Name(resp.remove_gpu_result)}")
        retry = svc.cfg.lease_retry_s
        for uid in due:
            self._retry_after[uid] = time.time() + retry
        svc.notify.event(pod, "GPULeaseExpired",
                         f"lease over but the GPUs are still in use "
                         f"({api.RemoveGPUResponse.RemoveGPUResult.Name(resp.remove_gpu_result)}"
                         f"); retrying every {retry:g} s (lease_force=false)", warning=True)
        if not self._stopped:
            old = self._retry_timers.pop((ns, name), None)
            if old is not None:
                old.cancel()
            self._retry_timers[(ns, name)] = asyncio.get_running_loop().call_later(
                retry, self._spawn, ns, name)
