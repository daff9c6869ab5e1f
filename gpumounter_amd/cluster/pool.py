"""Warm placeholder pool: pre-admitted GPUs that an attach claims with a metadata patch.

Attach latency in a real cluster is dominated by what happens *between* creating a placeholder
and reading its device IDs: scheduling, kubelet admission, the device plugin's Allocate — tens of
milliseconds even when images are cached, and seconds for the reference (``alpine:latest`` pulled
with policy Always). With ``warm_pool_size = K`` each worker keeps K single-GPU
*standby* placeholders admitted on its node. Those GPUs are held in the scheduler's books exactly
like any hot-mounted GPU (the ledger stays consistent), but belong to no tenant. An attach then:

1. picks the best standby GPUs for the pod with the xGMI/NUMA policy,
2. re-labels those placeholders to the pod (one PATCH each, in parallel) — no scheduling, no
   admission, no image pull,
3. mounts them; a detach hands them back to the pool (PATCH) and the pool tops itself up in the
   background.
Entire mounts claim K standby placeholders as one group (``gpumounter.amd.com/group``) and keep
the reference's all-or-nothing add/remove semantics. When the pool cannot cover a request the
worker falls back to creating placeholders as usual.

Priority. A claimed standby books a GPU its new tenant uses, so it must rank at least as high as
that tenant (cluster/placeholder.py ``priority_for``); a Pod's priority is immutable, so only
standbys created at that rank or higher can be claimed. By default standbys get the same floor
class as every placeholder (``placeholder_priority_class``): they cannot be preempted, and every
claim keeps the pool's latency. With a lower ``pool_priority_class`` idle standbys are
preemptible by higher-priority Pods (the scheduler evicts them, the pool refills when capacity
frees), and an attach that needs their GPUs *yields* them (:meth:`yield_low`: a conditional
DELETE while still standby) and books the GPUs with placeholders at tenant priority — the cold
path's latency, never a GPU held by a placeholder that ranks below its tenant.
"""
from __future__ import annotations

import asyncio
import secrets
import time
from typing import Awaitable, Callable, Dict, List, Optional, Sequence, Tuple

from gpumounter_amd.cluster.kube import Conflict, NotFound
from gpumounter_amd.cluster.placeholder import (ANN_GPUS, STANDBY_PREFIX, InsufficientGPU,
                                                LABEL_NODE, Placeholder,
                                                PlaceholderManager, Reservation,
                                                _label_value)
from gpumounter_amd.hw import topology
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.device import AmdGpu, normalize_device_id
from gpumounter_amd.models.types import (ANN_ATTACH_ID, ANN_CANDIDATE, ANN_CONTAINER, ANN_GROUP,
                                         ANN_IDEMPOTENCY, ANN_LEASE, ANN_MOUNT_MODE,
                                         ANN_OWNER_NAME, ANN_OWNER_UID, LABEL_APP,
                                         LABEL_APP_VALUE, LABEL_OWNER, LABEL_OWNER_NS,
                                         MODE_STANDBY)
from gpumounter_amd.utils import calls, log, trace

_log = log.get("cluster.pool")


class ClaimTaken(Exception):
    """The standby placeholder was claimed (or deleted) by someone else since it was chosen."""


def is_standby(p: dict) -> bool:
    return (p["metadata"].get("annotations") or {}).get(ANN_MOUNT_MODE) == MODE_STANDBY


class WarmPool:
    ALLOCATABLE_TTL_S = 30.0

    def __init__(self, cfg, ph: PlaceholderManager, inv, metrics=None) -> None:
        self.cfg = cfg
        self.ph = ph
        self.inv = inv
        self.metrics = metrics
        self.target = cfg.warm_pool_size
        self._lock = asyncio.Lock()          # serializes claims and give-backs on this node
        self._claimed: set = set()           # uids claimed but not yet visible as claimed
        self._refill_task: Optional[asyncio.Task] = None
        self._wake: Optional[asyncio.Event] = None
        self.exhausted = False               # last refill hit InsufficientGPU
        self._alloc_cache: Optional[tuple] = None   # (monotonic time, allocatable IDs)
        self._creating = 0        # standby placeholders a refill is about to create
        self._stopping = False
        # awaited before each refill (the worker sets Notifier.quiet): the POST and the
        # admission of a new standby wait until no attach/detach is in flight, instead of
        # sharing the worker's loop with the attach that emptied the pool
        self.quiet: Optional[Callable[[], Awaitable[None]]] = None
        # UIDs of the node's Pods the apiserver still has (the worker sets it): a checkpoint
        # entry of any other Pod is one being torn down, whose GPUs the next Allocate frees
        self.live_uids: Optional[Callable[[], set]] = None

    @property
    def enabled(self) -> bool:
        return self.target > 0

    # ------------------------------------------------------------------------ state
    def standby(self, min_priority: Optional[int] = None) -> List[Placeholder]:
        """Admitted standby placeholders (device IDs known); ``min_priority``: only those that
        rank at least that high (claimable by a tenant whose placeholders need that rank)."""
        out = []
        for p in self.ph.live():
            if not is_standby(p) or p["metadata"].get("uid") in self._claimed:
                continue
            if min_priority is not None and podu.priority_of(p) < min_priority:
                continue
            c = self.ph.cached(p)
            if c is None:
                ids = self.ph.last_ledger.get((p["metadata"]["namespace"],
                                               p["metadata"]["name"]))
                if not ids:
                    continue
                c = PlaceholderManager.from_pod(p, self.ph.last_ledger)
                self.ph.device_ids[c.uid] = c.device_ids
            out.append(c)
        return out

    def pending(self) -> int:
        return sum(1 for p in self.ph.live() if is_standby(p)
                   and podu.phase_of(p) != "Failed"
                   and self.ph.cached(p) is None
                   and not self.ph.last_ledger.get((p["metadata"]["namespace"],
                                                    p["metadata"]["name"])))

    def refilling(self) -> bool:
        """Standby placeholders are being created or admitted (they hold GPUs already)."""
        return self._creating > 0 or self.pending() > 0

    async def admitted(self, timeout: float) -> bool:
        """Wait, at most ``timeout``, until no standby placeholder is being created or
        admitted; True if the pool then has standby GPUs to claim."""
        end = time.monotonic() + timeout
        while self.refilling() and time.monotonic() < end:
            await asyncio.sleep(0.005)
        return bool(self.standby())

    # ------------------------------------------------------------------------ refill
    def standby_body(self) -> dict:
        name = f"{STANDBY_PREFIX}{_label_value(self.ph.node)[:40]}-{secrets.token_hex(4)}"
        body = self.ph.build({"metadata": {"name": "standby", "namespace": "", "uid": ""}},
                             1, MODE_STANDBY)
        pclass, _ = self.ph.standby_class()
        if pclass:
            body["spec"]["priorityClassName"] = pclass
        else:
            body["spec"].pop("priorityClassName", None)
        md = body["metadata"]
        md["name"] = name
        md["namespace"] = self.cfg.pool_namespace
        md["labels"] = {LABEL_APP: LABEL_APP_VALUE, LABEL_NODE: _label_value(self.ph.node)}
        md["annotations"] = {ANN_MOUNT_MODE: MODE_STANDBY, ANN_GPUS: "1"}
        md.pop("ownerReferences", None)
        for rc in body["spec"].get("resourceClaims") or []:     # DRA mode: its own claim
            rc["resourceClaimName"] = name
        return body

    async def start(self) -> None:
        if not self.enabled:
            return
        self._wake = asyncio.Event()
        self._refill_task = asyncio.ensure_future(self._refill_loop())
        self._wake.set()

    async def stop(self) -> None:
        self._stopping = True
        if self._refill_task is not None:
            self._refill_task.cancel()
            try:
                await self._refill_task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass

    # refill retries after a kubelet refused standbys at admission (a teardown in flight)
    REFUSED_RETRY_S = (0.1, 0.3, 1.0, 3.0)
    _refused = 0
    refusals = 0              # standby refills the kubelet refused (a running count)

    def poke(self) -> None:
        self._refused = 0            # news of capacity: a refusal gets its retries again
        self._wake_retry()

    def _wake_retry(self) -> None:
        if self._wake is not None:
            self._wake.set()

    async def _refill_loop(self) -> None:
        calls.mark_background()
        while not self._stopping:
            await self._wake.wait()
            self._wake.clear()
            try:
                if self.quiet is not None:
                    await self.quiet()
                await self.refill()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                _log.warning("pool refill failed: %s", e)
                await asyncio.sleep(1.0)
                self._wake.set()

    async def refill(self) -> int:
        """Create standby placeholders until ``target`` are admitted or pending."""
        # standbys the kubelet refused at admission (placeholder_binding=direct on a full node;
        # their refill's worker died before it could drop them): terminal, they hold nothing
        failed = [PlaceholderManager.from_pod(p, {}) for p in self.ph.live()
                  if is_standby(p) and podu.phase_of(p) == "Failed"]
        if failed:
            for ph in failed:
                ph.owner_uid, ph.attach_id = "", ""
            await self.ph.release(failed)
        missing = self.target - len(self.standby()) - self.pending()
        if missing <= 0:
            return 0
        # only ask for what the node can actually admit (allocatable − allocated). Allocated
        # comes from the device-manager checkpoint when it is in use, counting only Pods the
        # apiserver still has (a deleted Pod's entry lingers there until the kubelet's next
        # Allocate, which frees it; one still being torn down gets a standby refused, and the
        # refill looks again shortly), else from PodResources; the allocatable set changes only
        # with the plugin's device list and is re-read every ALLOCATABLE_TTL_S
        ck = self.ph.checkpoint
        snap = ck.snapshot() if ck is not None and ck.trusted else None
        if snap is not None:
            live = self.live_uids() if self.live_uids is not None else None
            allocated = {normalize_device_id(d) for uid, ids in snap.items()
                         if live is None or uid in live for d in ids}
        else:
            led = await self.ph.ledger.by_pod()
            self.ph.last_ledger = led
            allocated = {normalize_device_id(d) for ids in led.values() for d in ids}
        now = time.monotonic()
        if self._alloc_cache is None or now - self._alloc_cache[0] > self.ALLOCATABLE_TTL_S:
            self._alloc_cache = (now, await self.ph.ledger.allocatable())
        alloc = self._alloc_cache[1]
        if alloc is None:
            alloc = [g.bdf for g in self.inv.gpus()]
        free = sum(1 for d in alloc if normalize_device_id(d) not in allocated)
        # recount after the awaits above: a give-back may have refilled the pool meanwhile
        missing = min(self.target - len(self.standby()) - self.pending(), free)
        if missing <= 0:
            self.exhausted = True
            return 0
        created = []
        self._creating = missing       # counted by give_back until they exist (pending())
        try:
            for _ in range(missing):
                body = self.standby_body()
                try:
                    if self.ph.dra:                     # its ResourceClaim first
                        await self.ph._create_claims([body])  # noqa: SLF001
                    epoch = self.ph.informer.epoch
                    pod = await self.ph.create_pod(body)
                except Exception as e:  # noqa: BLE001
                    _log.warning("standby create failed: %s", e)
                    if self.ph.dra:     # unless the create happened after all (see there)
                        await self.ph._delete_unused_claims(  # noqa: SLF001
                            [(self.cfg.pool_namespace, body["metadata"]["name"])])
                    break
                self.ph.informer.upsert(pod, epoch)  # pending() counts it from here on
                self._creating -= 1
                md = pod["metadata"]
                created.append(Placeholder(md["namespace"], md["name"], md["uid"], (),
                                           MODE_STANDBY))
        finally:
            self._creating = 0
        if not created:
            return 0
        try:
            await self.ph._await_admission(created, self.cfg.attach_timeout_s)  # noqa: SLF001
            self.exhausted = False
            self._refused = 0
        except InsufficientGPU as e:
            # the node is full: drop the standby placeholders that could not be admitted
            self.exhausted = True
            unadmitted = [c for c in created if not c.device_ids]
            await self.ph.release(unadmitted)
            if str(e).startswith(("UnexpectedAdmissionError", "OutOf")):
                # refused by the kubelet, not the scheduler: it still counts GPUs of Pods
                # deleted a moment ago (their teardown frees them without any event we see),
                # so look again shortly rather than at the next capacity event
                self.refusals += 1
                if self._refused < len(self.REFUSED_RETRY_S):
                    delay = self.REFUSED_RETRY_S[self._refused]
                    self._refused += 1
                    asyncio.get_running_loop().call_later(delay, self._wake_retry)
        await self.ph.informer.poke()
        return len(created)

    # ------------------------------------------------------------------------ claim / return
    async def claim(self, owner: dict, n: int, entire: bool, attached: Sequence[AmdGpu],
                    attach_id: str = "", container: str = "",
                    idempotency_key: str = "",
                    want: Optional[Sequence[int]] = None,
                    lease_expires: float = 0.0,
                    min_priority: Optional[int] = None) -> Optional[Reservation]:
        """Claim ``n`` standby GPUs for ``owner`` (exactly the GPU indices ``want`` when the
        caller planned the placement over standby ∪ free GPUs); None if the pool cannot.
        ``min_priority``: only standbys that rank at least that high (the owner's placeholder
        rank, see the module docstring).
        ``lease_expires`` goes into the same conditional claim PATCH, so a leased claim is
        never recorded without its lease (and an unleased one clears any earlier owner's)."""
        async with self._lock:
            pool = self.standby(min_priority)
            if len(pool) < n:
                return None
            keys = self.inv.by_key()
            by_gpu: Dict[int, Placeholder] = {}
            cands: List[AmdGpu] = []
            for ph in pool:
                g = keys.get(normalize_device_id(ph.device_ids[0]))
                if g is not None:
                    by_gpu[g.index] = ph
                    cands.append(g)
            if want is not None:
                if len(want) != n or any(i not in by_gpu for i in want):
                    return None
                chosen = [by_gpu[i] for i in want]
            else:
                plc = topology.choose(cands, n, self.inv.links(), attached=attached,
                                      policy=self.cfg.topology_policy)
                if plc is None:
                    return None
                chosen = [by_gpu[i] for i in plc.chosen]
            mode = "entire" if entire else "single"
            group = secrets.token_hex(4) if entire else ""
            patch = {"metadata": {
                "labels": {LABEL_OWNER: _label_value(podu.name_of(owner)),
                           LABEL_OWNER_NS: _label_value(podu.ns_of(owner))},
                "annotations": {ANN_OWNER_UID: podu.uid_of(owner),
                                ANN_OWNER_NAME: podu.name_of(owner), ANN_MOUNT_MODE: mode,
                                ANN_ATTACH_ID: attach_id, ANN_CONTAINER: container,
                                ANN_IDEMPOTENCY: idempotency_key or None,
                                ANN_GROUP: group or None, ANN_CANDIDATE: None,
                                ANN_LEASE: f"{lease_expires:.3f}" if lease_expires > 0
                                else None}}}
            for ph in chosen:
                self._claimed.add(ph.uid)
            seen = self._versions()
            with trace.span("pool_claim", placeholders=len(chosen)):
                epoch = self.ph.informer.epoch
                res = await asyncio.gather(
                    *[self._claim_one(ph, patch, seen.get(ph.uid), attach_id) for ph in chosen],
                    return_exceptions=True)
            ok = [r for r in res if isinstance(r, dict)]
            for r in ok:
                self.ph.informer.upsert(r, epoch)
            for ph in chosen:
                self._claimed.discard(ph.uid)
            if len(ok) != len(chosen):
                # undo the partial claim, then let the caller fall back. A PATCH that failed may
                # still have taken effect (its reply lost), so every chosen placeholder that is
                # this attach's goes back; one that cannot be put back is deleted — the caller
                # never mounts these, and a claim left standing would give the owner a GPU it
                # was told it did not get. One another claim took is left to its owner.
                taken = [ph for ph, r in zip(chosen, res) if isinstance(r, ClaimTaken)]
                mine = [ph for ph in chosen if ph not in taken]
                back, theirs = await self._unclaim(mine, attach_id)
                stray = [ph for ph in mine if ph not in back and ph not in theirs]
                if taken:
                    _log.info("standby placeholder(s) %s claimed elsewhere; falling back",
                              [ph.name for ph in taken])
                if stray:
                    for ph in stray:            # deleted only while still this attach's
                        ph.owner_uid, ph.attach_id = podu.uid_of(owner), attach_id
                    await self.ph.release(stray)
                return None
            for ph in chosen:
                ph.mode = mode
                ph.owner_uid, ph.attach_id = podu.uid_of(owner), attach_id
            _log.debug("claimed %s for %s/%s attach %s", [ph.name for ph in chosen],
                       podu.ns_of(owner), podu.name_of(owner), attach_id)
            if self.metrics is not None:
                self.metrics.reconcile_actions.labels(action="pool_claim").inc(len(chosen))
        self.poke()
        return Reservation(chosen)

    async def cancel_pending_low(self, min_priority: int) -> int:
        """Delete standby placeholders that rank below ``min_priority`` and are not admitted
        yet (a refill in flight): their GPUs look free to an attach at that rank, which would
        then lose the race for them to a standby it cannot claim. Returns how many."""
        async with self._lock:
            pend = [PlaceholderManager.from_pod(p, {}) for p in self.ph.live()
                    if is_standby(p) and podu.priority_of(p) < min_priority
                    and self.ph.cached(p) is None
                    and not self.ph.last_ledger.get((p["metadata"]["namespace"],
                                                     p["metadata"]["name"]))]
            if not pend:
                return 0
            for ph in pend:
                ph.owner_uid, ph.attach_id = "", ""
            try:
                await self.ph.release(pend)
            except Exception as e:  # noqa: BLE001 - the attach's own retry covers the rest
                _log.warning("cancelling pending standby placeholders: %s", e)
            return len(pend)

    async def yield_low(self, n: int, min_priority: int, attached: Sequence[AmdGpu] = ()
                        ) -> List[Placeholder]:
        """Give up to ``n`` standby GPUs that rank below ``min_priority`` back to the scheduler
        (DELETE, conditional on each still being standby), so an attach at that rank can book
        them with placeholders of its own; the best-placed ones for ``attached`` go first.
        Returns those released. The pool refills later from whatever is free then."""
        async with self._lock:
            low = [ph for ph in self.standby() if ph.priority < min_priority]
            if not low or n <= 0:
                return []
            keys = self.inv.by_key()
            by_gpu = {}
            for ph in low:
                g = keys.get(normalize_device_id(ph.device_ids[0]))
                if g is not None:
                    by_gpu[g.index] = ph
            k = min(n, len(low))
            plc = topology.choose([keys[normalize_device_id(ph.device_ids[0])]
                                   for ph in by_gpu.values()], k, self.inv.links(),
                                  attached=attached, policy=self.cfg.topology_policy) \
                if len(by_gpu) >= k else None
            chosen = [by_gpu[i] for i in plc.chosen] if plc is not None else low[:k]
            for ph in chosen:
                ph.owner_uid, ph.attach_id = "", ""     # released only while still standby
            with trace.span("pool_yield", placeholders=len(chosen)):
                try:
                    await self.ph.release(chosen)
                except Exception as e:  # noqa: BLE001 - what was released still counts
                    _log.warning("yielding standby placeholders: %s", e)
            gone = [ph for ph in chosen if (ph.namespace, ph.name) not in self.ph.informer.cache
                    or ph.uid in self.ph.tombstones]
            if self.metrics is not None and gone:
                self.metrics.reconcile_actions.labels(action="pool_yield").inc(len(gone))
            _log.info("yielded %d low-priority standby GPU(s) to an attach at priority %d",
                      len(gone), min_priority)
            return gone

    def _versions(self) -> Dict[str, str]:
        """uid → resourceVersion of every standby placeholder as the informer last saw it."""
        return {p["metadata"]["uid"]: p["metadata"].get("resourceVersion", "")
                for p in self.ph.live() if is_standby(p)}

    @staticmethod
    def _mine(pod: dict, attach_id: str) -> bool:
        return bool(attach_id) and \
            (pod["metadata"].get("annotations") or {}).get(ANN_ATTACH_ID) == attach_id

    async def _claim_one(self, ph: Placeholder, patch: dict, rv: Optional[str],
                         attach_id: str) -> dict:
        """Claim one standby placeholder with a merge patch that carries the resourceVersion
        the choice was made on: it applies only if nothing changed the placeholder since. The
        informer can be behind the apiserver (after a relist an acknowledged write is not in the
        cache yet; a worker killed mid-claim may still have a PATCH in flight), and an
        unconditional claim of a placeholder that is no longer standby hands one GPU to two
        Pods. On a conflict the placeholder is read back: this attach's own claim (an earlier
        attempt whose reply was lost) counts as done, one still standby is claimed at its new
        version, anything else raises :class:`ClaimTaken`."""
        kube = self.ph.kube
        for _ in range(3):
            if not rv:
                cur = await kube.get_pod(ph.namespace, ph.name)
                if not self._claimable(cur, ph):
                    raise ClaimTaken(ph.name)
                rv = cur["metadata"]["resourceVersion"]
            try:
                return await kube.patch_pod(ph.namespace, ph.name, {
                    "metadata": dict(patch["metadata"], resourceVersion=rv)})
            except NotFound:
                raise ClaimTaken(ph.name) from None
            except Conflict:
                cur = await kube.get_pod(ph.namespace, ph.name)
                if cur["metadata"].get("uid") == ph.uid and self._mine(cur, attach_id):
                    return cur
                if not self._claimable(cur, ph):
                    raise ClaimTaken(ph.name) from None
                rv = cur["metadata"]["resourceVersion"]
        raise ClaimTaken(ph.name)

    @staticmethod
    def _claimable(pod: dict, ph: Placeholder) -> bool:
        md = pod["metadata"]
        return md.get("uid") == ph.uid and is_standby(pod) and not md.get("deletionTimestamp")

    async def _unclaim(self, phs: Sequence[Placeholder], attach_id: str
                       ) -> Tuple[List[Placeholder], List[Placeholder]]:
        """Undo a failed claim: put back into the pool each placeholder this attach claimed.
        Returns (free again, not this attach's to undo); the rest could not be read or put
        back."""
        res = await asyncio.gather(*[self._put_back(ph, lambda cur: self._mine(cur, attach_id))
                                     for ph in phs], return_exceptions=True)
        return self._sort_back(phs, res)

    def _sort_back(self, phs, res) -> Tuple[List[Placeholder], List[Placeholder]]:
        back, theirs = [], []
        for ph, r in zip(phs, res):
            if r is True:
                back.append(ph)
            elif r is False:
                theirs.append(ph)
            else:
                _log.error("return %s/%s to pool: %s", ph.namespace, ph.name, r)
        return back, theirs

    @staticmethod
    def _standby_patch(rv: Optional[str]) -> dict:
        return {"metadata": {
            "labels": {LABEL_OWNER: None, LABEL_OWNER_NS: None},
            "annotations": {ANN_OWNER_UID: None, ANN_OWNER_NAME: None,
                            ANN_MOUNT_MODE: MODE_STANDBY, ANN_ATTACH_ID: None,
                            ANN_CONTAINER: None, ANN_GROUP: None, ANN_IDEMPOTENCY: None,
                            # surplus of a trim/correction pick comes back as candidates: a
                            # claimed one still marked would be invisible to its new owner's
                            # ledger view, and released under it as an abandoned pick
                            ANN_CANDIDATE: None,
                            # an earlier owner's lease would expire the next owner's GPU
                            ANN_LEASE: None},
            # only at a version read while the placeholder was still the caller's
            "resourceVersion": rv}}

    async def _put_back(self, ph: Placeholder, ours: Callable[[dict], bool],
                        rv: Optional[str] = None) -> bool:
        """Return one placeholder to the pool with a merge patch conditional on a version at
        which it was still ``ours``, so one that someone else has claimed since is never taken
        from them. True: standby now; False: not ours (left alone). Raises when it could not
        be read or written."""
        for _ in range(3):
            if not rv:
                try:
                    cur = await self.ph.kube.get_pod(ph.namespace, ph.name)
                except NotFound:
                    return False                        # gone: nothing left to return
                if cur["metadata"].get("uid") != ph.uid or not ours(cur):
                    return self._claimable(cur, ph)     # already standby counts as back
                rv = cur["metadata"]["resourceVersion"]
            epoch = self.ph.informer.epoch
            try:
                r = await self.ph.kube.patch_pod(ph.namespace, ph.name, self._standby_patch(rv))
            except NotFound:
                return False
            except Conflict:
                rv = None                               # changed since: read it again
                continue
            self.ph.informer.upsert(r, epoch)
            _log.debug("returned %s to the pool (was %s)", ph.name, ph.owner_uid or "?")
            return True
        raise Conflict(409, f"{ph.name} kept changing while being returned to the pool")

    async def give_back(self, phs: Sequence[Placeholder]) -> None:
        """Return detached placeholders to the pool (up to ``target``); delete the rest. Each
        goes back only at a version at which it has the owner the caller's view showed
        (``Placeholder.owner_uid``): one put back and claimed anew meanwhile stays with its new
        owner."""
        async with self._lock:
            # standby being admitted count too, or a refill racing a give-back overfills
            room = max(self.target - len(self.standby()) - self.pending() - self._creating, 0)
            # with a low pool class, a placeholder that booked a tenant's GPU (at tenant rank)
            # does not become an idle standby: standbys must stay preemptible. It is deleted
            # and the refill creates a standby at the pool's class
            cap = self.ph.standby_class()[1] if getattr(self.cfg, "pool_priority_class", "") \
                else None
            keep = [p for p in phs if p.device_ids and len(p.device_ids) == 1
                    and (cap is None or p.priority <= cap)][:room]
            drop = [p for p in phs if p not in keep]
            cache = {p["metadata"]["uid"]: p for p in self.ph.live()}

            def put(ph: Placeholder):
                # at the cached version if the cache agrees it has the holder the caller's view
                # showed, else at a version read now
                seen = cache.get(ph.uid)
                rv = seen["metadata"].get("resourceVersion") \
                    if seen is not None and ph.held_by_me(seen) else None
                return self._put_back(ph, ph.held_by_me, rv)
            with trace.span("pool_return", placeholders=len(keep)):
                res = await asyncio.gather(*[put(ph) for ph in keep], return_exceptions=True)
            back, theirs = self._sort_back(keep, res)
            drop += [p for p in keep if p not in back and p not in theirs]
        if drop:
            await self.ph.release(drop)
        self.poke()
