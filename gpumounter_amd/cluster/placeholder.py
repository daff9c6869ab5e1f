"""Placeholder pods — the scheduler-consistent GPU ledger.

Reference: ``GetAvailableGPU`` creates ``total/perPod`` slave pods *sequentially* in ``gpu-pool``
(``alpine:latest`` sleep loop, ``nvidia.com/gpu`` limit, nodeSelector hostname, cross-namespace
controller ownerReference), busy-polls them until Running/Unschedulable, then reads their device
IDs from PodResources (reference: pkg/util/gpu/allocator/allocator.go:40-99,189-282). The GPU is
thereby held in the scheduler's books by a pod the scheduler knows about, while the tenant uses it.

Kept: the ledger model, the ``<owner>-slave-pod-<hex>`` naming, nodeSelector pinning, the
Unschedulable → InsufficientGPU mapping. Changed:

* creates run concurrently; readiness is awaited on a watch (no polling of the apiserver);
* the allocation is read as soon as the kubelet *admits* the placeholder (device-plugin Allocate
  happens at admission) instead of after the container is Running;
* a pre-pulled ``pause`` image with ``IfNotPresent`` (the reference's ``:latest`` forces a pull);
  ``terminationGracePeriodSeconds: 0`` (the reference's ``sh`` loop ignores SIGTERM, so every
  detach waited the default 30 s grace);
* owner matching is an exact label + UID annotation (the reference's substring match lets pod
  ``a`` see the slaves of ``xa`` and ignores namespaces — defect 3);
* in ``tenant`` namespace mode the ownerReference is same-namespace (valid for the garbage
  collector); in ``pool`` mode no cross-namespace ownerReference is written at all (Kubernetes
  ≥1.20 treats it as absent and deletes the placeholder — defect 4) and the reconciler collects
  placeholders whose owner is gone;
* the preferred (xGMI/NUMA-aware) device set is attached as an annotation for
  GetPreferredAllocation-capable device plugins, and any deviation is counted;
* ``reserve_trim`` enforces the placement whatever the device plugin picks: every free GPU is
  held by a 1-GPU placeholder at once, the topology-chosen subset is kept, the rest released;
* on DRA clusters (``gpu_allocation=dra``) a placeholder holds a ResourceClaim of its own name
  instead of an extended-resource limit, and the topology-chosen devices are a CEL selector of
  that claim: the scheduler allocates exactly them (no trim needed). If they were taken
  meanwhile, the reservation is retried once without the selector;
* a placeholder never ranks below the tenant whose GPU it books (:meth:`priority_for`): the
  reference's slave pods have priority 0, so any higher-priority Pod requesting a GPU on a
  full node makes the scheduler preempt one, and the GPU is revoked under a running job.
  Placeholders get the floor class ``placeholder_priority_class`` (shipped: value 1000000,
  ``preemptionPolicy: Never``, so they never preempt anyone either), or the tenant's own class
  when the tenant ranks higher.
"""
from __future__ import annotations

import asyncio
import contextlib
import secrets
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from gpumounter_amd.cluster.informer import PodInformer
from gpumounter_amd.cluster.kube import ApiError, Conflict, KubeClient, NotFound
from gpumounter_amd.cluster.quota import QuotaExceeded
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.types import (ANN_ATTACH_ID, ANN_CANDIDATE, ANN_CONTAINER, ANN_GROUP,
                                         ANN_IDEMPOTENCY, ANN_INCARNATION, ANN_LEASE,
                                         ANN_MOUNT_MODE, ANN_OWNER_UID, ANN_PREFERRED, LABEL_APP,
                                         LABEL_APP_VALUE, LABEL_OWNER, LABEL_OWNER_NS,
                                         SLAVE_SUFFIX)
from gpumounter_amd.node.ledger import LedgerClient
from gpumounter_amd.utils import calls, log, trace

_log = log.get("cluster.placeholder")
LABEL_NODE = "gpumounter.amd.com/node"
# number of GPUs a placeholder holds (DRA mode: there is no extended-resource limit to read)
ANN_GPUS = "gpumounter.amd.com/gpus"
CLAIM_REQUEST = "gpus"
# warm-pool placeholders (cluster/pool.py) change hands: claimed by a Pod, given back, claimed
# by another
STANDBY_PREFIX = "gpumounter-standby-"


# the Priority admission plugin's refusal of a class that does not exist
_NO_CLASS = "no PriorityClass with name"


class Reowned(Exception):
    """A pool placeholder that changed owner since the caller decided to release it."""


class InsufficientGPU(RuntimeError):
    pass


class ReserveError(RuntimeError):
    pass


@dataclass
class Placeholder:
    namespace: str
    name: str
    uid: str = ""
    device_ids: Tuple[str, ...] = ()
    mode: str = "single"
    candidate: bool = False      # held by a trim/correction pick, not yet confirmed
    # the holder as the view this object came from shows it: the owner Pod's uid ("" = none:
    # standby) and the attach that claimed or created it. A warm-pool placeholder changes hands,
    # also back to the same Pod by a later attach; its release applies only while it still has
    # this holder (see _delete)
    owner_uid: str = ""
    attach_id: str = ""
    priority: int = 0            # spec.priority (immutable for the Pod's lifetime)

    def held_by_me(self, pod: dict) -> bool:
        """``pod`` (the placeholder as the apiserver has it) still has this object's holder."""
        ann = pod["metadata"].get("annotations") or {}
        return (ann.get(ANN_OWNER_UID) or "") == self.owner_uid and \
            (not self.attach_id or (ann.get(ANN_ATTACH_ID) or "") == self.attach_id)


@dataclass
class Reservation:
    placeholders: List[Placeholder] = field(default_factory=list)
    # the device set placement asked for (empty: no preference) — for the mismatch metric
    preferred: List[str] = field(default_factory=list)
    # the device plugin chose these freely and other GPUs were free: placement may correct it
    corrigible: bool = False

    @property
    def device_ids(self) -> List[str]:
        return [d for p in self.placeholders for d in p.device_ids]


def _message(e: "ApiError") -> str:
    body = e.body
    if isinstance(body, dict):
        return str(body.get("message") or e)
    return str(body or e)


def _label_value(s: str) -> str:
    s = s[:63]
    return s.rstrip("-_.") or "x"


def _admitted(pod: Optional[dict]) -> bool:
    """The kubelet has run admission (device-plugin Allocate) for this pod: it posts container
    statuses (ContainerCreating) only afterwards."""
    return bool(pod) and (bool(pod.get("status", {}).get("containerStatuses")) or
                          podu.phase_of(pod) == "Running")


class PlaceholderManager:
    # admission re-read backoff when no placeholder event arrives: first wait, cap (seconds)
    ADMISSION_BACKOFF_S = (0.010, 0.100)
    # the same with the device-manager checkpoint in use: events (pod watch + inotify) carry
    # the normal path, the RPC is only a safety net
    ADMISSION_BACKOFF_CKPT_S = (0.050, 0.200)
    # consecutive "admitted per the apiserver, absent from the checkpoint" reads after which
    # the checkpoint counts as not maintained by this kubelet
    CHECKPOINT_MISSES = 3
    # how long a tombstone outlives its object in the cache: a relist whose list is older than
    # our delete still gets the DELETED event from the resumed watch (see _on_event)
    TOMBSTONE_KEEP_S = 60.0
    # conditional DELETEs of one placeholder before a release gives up (see _delete)
    DELETE_ATTEMPTS = 10

    def __init__(self, cfg, kube: KubeClient, ledger: LedgerClient, informer: PodInformer,
                 node_name: str, faults=None) -> None:
        from gpumounter_amd.utils.faults import NONE

        self.cfg = cfg
        self.kube = kube
        self.ledger = ledger
        self.informer = informer
        self.node = node_name
        self.faults = faults if faults is not None else NONE
        # the kubelet device manager's checkpoint (node/checkpoint.py), set by the worker when
        # ledger_source=auto: admission then needs no PodResources call
        self.checkpoint = None
        self.checkpoint_hits = 0
        self._checkpoint_misses = 0
        # uid → device IDs of admitted placeholders (immutable for a pod's lifetime)
        self.device_ids: Dict[str, Tuple[str, ...]] = {}
        # uids we deleted but the watch has not reported yet: excluded from every query, so a
        # released GPU is never seen as still attached (no need to wait for the DELETED event)
        self.tombstones: Dict[str, float] = {}
        self.incarnation = secrets.token_hex(6)     # this process (ANN_INCARNATION)
        informer.handlers.append(self._on_event)
        self.last_ledger: Dict[Tuple[str, str], List[str]] = {}
        # called with the placeholder pod when something other than us deletes it (kubectl,
        # eviction, preemption, namespace deletion): its GPU is going back to the scheduler
        self.on_foreign_delete: List[Callable[[dict], None]] = []
        self._foreign_seen: Dict[str, float] = {}
        self._bg: set = set()       # background claim deletions (DRA mode)
        # PriorityClass name → value; None: the class does not exist in the cluster. Read at
        # start (resolve_priority); a class missing at create time is marked here too
        self.class_values: Dict[str, Optional[int]] = {}
        self.priority_fallbacks = 0     # placeholders created without their floor class

    def _on_event(self, etype: str, pod: dict) -> None:
        md = pod.get("metadata", {})
        uid = md.get("uid", "")
        if (etype == "DELETED" or (etype == "MODIFIED" and md.get("deletionTimestamp"))) \
                and uid and uid not in self.tombstones and uid not in self._foreign_seen:
            self._foreign_seen[uid] = 0.0
            for cb in list(self.on_foreign_delete):
                try:
                    cb(pod)
                except Exception:  # noqa: BLE001
                    _log.exception("foreign-delete callback failed")
        if etype == "DELETED":
            self.tombstones.pop(uid, None)
            self.device_ids.pop(uid, None)
            self._foreign_seen.pop(uid, None)
        elif etype == "RELIST":
            live = {p["metadata"].get("uid") for p in self.informer.cache.values()}
            # the watch resumes from the list's version, which can be older than a delete of
            # ours: that DELETED event is still to come, and without its tombstone it reads as
            # a foreign delete (a revocation under the Pod). Tombstones of deletes the list
            # already left out go once they are old enough that no event for them is pending
            old = asyncio.get_running_loop().time() - self.TOMBSTONE_KEEP_S
            for uid in [u for u, t in self.tombstones.items() if u not in live and t < old]:
                self.tombstones.pop(uid, None)
            for uid in [u for u in self.device_ids if u not in live]:
                self.device_ids.pop(uid, None)
            for uid in [u for u in self._foreign_seen if u not in live]:
                self._foreign_seen.pop(uid, None)

    # ------------------------------------------------------------------------ priority
    async def resolve_priority(self) -> None:
        """Read the values of the configured classes (the floor, the pool's). A class the
        apiserver does not have is recorded as absent: placeholders then fall back to their
        tenant's class (still never below it) and the doctor reports the missing class."""
        names = {self.cfg.placeholder_priority_class,
                 getattr(self.cfg, "pool_priority_class", "")} - {""}
        for name in sorted(names):
            try:
                pc = await self.kube.get_priority_class(name)
                self.class_values[name] = int(pc.get("value", 0))
            except NotFound:
                self.class_values[name] = None
                _log.error("PriorityClass %s does not exist: placeholders fall back to their "
                           "tenant's priority (apply deploy/placeholder-priority.yaml)", name)
            except Exception as e:  # noqa: BLE001 - RBAC without priorityclasses: config value
                _log.info("PriorityClass %s not readable (%s); assuming value %d", name, e,
                          self.cfg.placeholder_priority_value)

    def class_value(self, name: str) -> Optional[int]:
        """Value of ``name``; the configured floor value when it could not be read."""
        if name in self.class_values:
            return self.class_values[name]
        if name == self.cfg.placeholder_priority_class:
            return int(self.cfg.placeholder_priority_value)
        return None

    def priority_for(self, owner: dict) -> Tuple[str, int]:
        """(priorityClassName, priority) of a placeholder that books a GPU for ``owner``:
        the floor class, or the owner's own class when the owner ranks higher (or when the
        floor is off or missing). Never below the owner."""
        spec = owner.get("spec") or {}
        o_cls, o_prio = spec.get("priorityClassName") or "", podu.priority_of(owner)
        floor = self.cfg.placeholder_priority_class
        fv = self.class_value(floor) if floor else None
        if fv is None or (o_prio > fv and getattr(self.cfg, "placeholder_priority_inherit",
                                                  True)):
            return o_cls, o_prio
        return floor, fv

    def standby_class(self) -> Tuple[str, int]:
        """(class, value) of warm-pool standby placeholders: ``pool_priority_class``, else the
        floor class; no class when the chosen one is missing."""
        name = getattr(self.cfg, "pool_priority_class", "") or \
            self.cfg.placeholder_priority_class
        v = self.class_value(name) if name else None
        return (name, v) if v is not None else ("", 0)

    def _class_missing(self, e: BaseException) -> Optional[str]:
        """The class a create failed on because it does not exist (None: another error)."""
        if isinstance(e, ApiError) and e.status == 403 and _NO_CLASS in _message(e):
            return _message(e).split(_NO_CLASS, 1)[1].split()[0]
        return None

    # ------------------------------------------------------------------------ spec
    def namespace_for(self, owner: dict) -> str:
        if self.cfg.placeholder_namespace_mode == "tenant":
            return podu.ns_of(owner)
        return self.cfg.pool_namespace

    @staticmethod
    def selector_for_node(node: str) -> str:
        return f"{LABEL_APP}={LABEL_APP_VALUE},{LABEL_NODE}={_label_value(node)}"

    def build(self, owner: dict, n_gpus: int, mode: str, preferred: Sequence[str] = (),
              attach_id: str = "", container: str = "", idempotency_key: str = "",
              lease_expires: float = 0.0) -> dict:
        """The placeholder Pod for ``owner``. ``lease_expires`` (Unix seconds, 0 = none) is
        written at creation, so a leased GPU is never booked without its lease (reference:
        every slave-pod field is set in the create, allocator.go:189-234)."""
        ns = self.namespace_for(owner)
        name = podu.name_of(owner)[: 253 - 20] + SLAVE_SUFFIX + secrets.token_hex(3)
        md = {
            "name": name,
            "namespace": ns,
            "labels": {LABEL_APP: LABEL_APP_VALUE,
                       LABEL_OWNER: _label_value(podu.name_of(owner)),
                       LABEL_OWNER_NS: _label_value(podu.ns_of(owner)),
                       LABEL_NODE: _label_value(self.node)},
            "annotations": {ANN_OWNER_UID: podu.uid_of(owner), ANN_MOUNT_MODE: mode,
                            ANN_ATTACH_ID: attach_id, ANN_CONTAINER: container,
                            ANN_INCARNATION: self.incarnation,
                            "gpumounter.amd.com/owner-name": podu.name_of(owner)},
        }
        if preferred:
            md["annotations"][ANN_PREFERRED] = ",".join(preferred)
        if idempotency_key:
            md["annotations"][ANN_IDEMPOTENCY] = idempotency_key
        if lease_expires > 0:
            md["annotations"][ANN_LEASE] = f"{lease_expires:.3f}"
        if ns == podu.ns_of(owner):
            md["ownerReferences"] = [{"apiVersion": "v1", "kind": "Pod",
                                      "name": podu.name_of(owner), "uid": podu.uid_of(owner),
                                      "controller": True, "blockOwnerDeletion": True}]
        spec = {
            "nodeSelector": {"kubernetes.io/hostname": self.node},
            "tolerations": [{"operator": "Exists"}],
            "terminationGracePeriodSeconds": 0,
            "automountServiceAccountToken": False,
            "enableServiceLinks": False,
            "restartPolicy": "Always",
            "containers": [{
                "name": "gpu-holder",
                "image": self.cfg.placeholder_image,
                "imagePullPolicy": self.cfg.placeholder_pull_policy,
                "resources": {"limits": {self.cfg.resource_name: str(n_gpus)},
                              "requests": {"cpu": "1m", "memory": "4Mi"}},
            }],
        }
        md["annotations"][ANN_GPUS] = str(n_gpus)
        if self.direct:
            spec["nodeName"] = self.node        # the kubelet admits it; no scheduling cycle
        if self.dra:
            res = spec["containers"][0]["resources"]
            res.pop("limits")
            res["claims"] = [{"name": CLAIM_REQUEST}]
            spec["resourceClaims"] = [{"name": CLAIM_REQUEST, "resourceClaimName": name}]
        pclass, _ = self.priority_for(owner)
        if pclass:
            spec["priorityClassName"] = pclass
        return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec}

    @property
    def reownable(self) -> bool:
        """Placeholders can change holder (warm-pool claims and give-backs, cluster/pool.py)."""
        return getattr(self.cfg, "warm_pool_size", 0) > 0

    @property
    def direct(self) -> bool:
        """Placeholders are bound to this node at creation (placeholder_binding=direct)."""
        return getattr(self.cfg, "placeholder_binding", "scheduler") == "direct"

    @property
    def dra(self) -> bool:
        return getattr(self.cfg, "gpu_allocation", "device-plugin") == "dra"

    def claim_for(self, body: dict) -> dict:
        """The ResourceClaim a DRA-mode placeholder references: ``count`` devices of the GPU
        device class, narrowed to the preferred devices (by PCI address) when there are any."""
        md = body["metadata"]
        ann = md.get("annotations") or {}
        n = int(ann.get(ANN_GPUS, "1"))
        exactly = {"deviceClassName": self.cfg.dra_device_class,
                   "allocationMode": "ExactCount", "count": n}
        pref = [d for d in ann.get(ANN_PREFERRED, "").split(",") if d]
        if pref and len(pref) == n:
            vals = ", ".join(f'"{d}"' for d in pref)
            exactly["selectors"] = [{"cel": {"expression":
                f'device.attributes["{self.cfg.dra_driver}"].{self.cfg.dra_bdf_attribute} '
                f'in [{vals}]'}}]
        return {"apiVersion": "resource.k8s.io/v1", "kind": "ResourceClaim",
                "metadata": {"name": md["name"], "namespace": md["namespace"],
                             "labels": dict(md.get("labels") or {}),
                             "annotations": {ANN_OWNER_UID: ann.get(ANN_OWNER_UID, "")}},
                "spec": {"devices": {"requests": [{"name": CLAIM_REQUEST, "exactly": exactly}]}}}

    # ------------------------------------------------------------------------ queries
    def live(self) -> List[dict]:
        """Placeholders on this node that are neither terminating nor released by us."""
        return self.informer.list(lambda p: not p["metadata"].get("deletionTimestamp")
                                  and p["metadata"].get("uid") not in self.tombstones)

    def owned_by(self, owner: dict, candidates: bool = False) -> List[dict]:
        """The owner's placeholders; ``candidates``: also those a trim/correction pick holds
        and has not confirmed (never mounted; released by the pick or the reconciler)."""
        uid = podu.uid_of(owner)
        oname, ons = _label_value(podu.name_of(owner)), _label_value(podu.ns_of(owner))

        def mine(p: dict) -> bool:
            md = p["metadata"]
            lab = md.get("labels") or {}
            ann = md.get("annotations") or {}
            return (lab.get(LABEL_OWNER) == oname and lab.get(LABEL_OWNER_NS) == ons
                    and ann.get(ANN_OWNER_UID) == uid
                    and (candidates or ANN_CANDIDATE not in ann)
                    and not md.get("deletionTimestamp")
                    and md.get("uid") not in self.tombstones)

        return self.informer.list(mine)

    # ------------------------------------------------------------------------ reserve
    async def reserve(self, owner: dict, total: int, entire: bool, preferred: Sequence[str] = (),
                      attach_id: str = "", container: str = "",
                      idempotency_key: str = "", lease_expires: float = 0.0) -> Reservation:
        """Entire mount = one placeholder holding ``total`` GPUs (all-or-nothing at the
        scheduler, reference QuickStart.md:52); single mount = ``total`` placeholders × 1 GPU."""
        if total <= 0:
            raise ValueError(f"bad reservation size {total}")
        per_pod = total if entire else 1
        k = total // per_pod
        mode = "entire" if entire else "single"
        prefs = [list(preferred[i * per_pod:(i + 1) * per_pod]) for i in range(k)] \
            if len(preferred) == total else [[] for _ in range(k)]
        bodies = [self.build(owner, per_pod, mode, prefs[i], attach_id, container,
                             idempotency_key, lease_expires) for i in range(k)]
        created = await self._create(bodies, owner)
        try:
            with trace.span("placeholder_wait"):
                self.faults.check("placeholder_wait")
                await self._await_admission(created, self.cfg.attach_timeout_s)
                self.faults.check("placeholder_wait", "after")
        except InsufficientGPU:
            await self.release(created)
            if not (self.dra and len(preferred) == total):
                raise
            # DRA selectors are hard constraints: the chosen devices went to someone else
            # since our ledger view; any free ones will do
            _log.info("preferred devices %s not allocatable; retrying unpinned",
                      list(preferred))
            return await self.reserve(owner, total, entire, (), attach_id, container,
                                      idempotency_key, lease_expires)
        except BaseException:
            await self.release(created)
            raise
        return Reservation(created)

    async def hold_singles(self, owner: dict, width: int, entire: bool, group: str = "",
                           attach_id: str = "", container: str = "",
                           idempotency_key: str = "", lease_expires: float = 0.0
                           ) -> List[Placeholder]:
        """Create ``width`` 1-GPU placeholders at once and wait for their admission; returns
        the admitted ones (those the scheduler could not place are released). An entire mount
        ties them by ``group`` (``ANN_GROUP``)."""
        if width <= 0:
            return []
        mode = "entire" if entire else "single"
        bodies = [self.build(owner, 1, mode, (), attach_id, container, idempotency_key,
                             lease_expires) for _ in range(width)]
        for b in bodies:
            b["metadata"]["annotations"][ANN_CANDIDATE] = attach_id or "1"
            if group:
                b["metadata"]["annotations"][ANN_GROUP] = group
        created = await self._create(bodies, owner)
        for p in created:
            p.candidate = True
        try:
            with trace.span("placeholder_wait"):
                self.faults.check("placeholder_wait")
                failed = await self._await_admission(created, self.cfg.attach_timeout_s,
                                                     tolerant=True)
                self.faults.check("placeholder_wait", "after")
        except BaseException:
            await self.release(created)
            raise
        if failed:
            try:
                await self.release(failed)
            except BaseException:
                # the caller never learns of the admitted ones either: let them go too (the
                # candidate mark leads the follow-up and the sweep to any this cannot delete)
                with contextlib.suppress(Exception):
                    await self.release([p for p in created if p not in failed])
                raise
        return [p for p in created if p not in failed]

    async def reserve_trim(self, owner: dict, total: int, entire: bool, width: int,
                           pick: Callable[[List[str]], Sequence[str]], attach_id: str = "",
                           container: str = "", idempotency_key: str = "",
                           lease_expires: float = 0.0
                           ) -> Tuple[Reservation, List[Placeholder]]:
        """Topology-pinned reservation. Which GPU the device plugin hands a
        placeholder is opaque to us, so hold ``width`` (= every free GPU) 1-GPU placeholders at
        once and keep the ``total`` whose device IDs ``pick`` returns. Returns the reservation and
        the surplus placeholders, which the caller releases (or returns to the warm pool).
        Entire mounts are the kept placeholders tied by one ``ANN_GROUP`` id, the same shape
        as a warm-pool entire claim."""
        if total <= 0 or width < total:
            raise ValueError(f"bad trim reservation {total}/{width}")
        admitted = await self.hold_singles(owner, width, entire,
                                           secrets.token_hex(4) if entire else "", attach_id,
                                           container, idempotency_key, lease_expires)
        if len(admitted) < total:
            await self.release(admitted)
            raise InsufficientGPU(f"only {len(admitted)} of {total} GPUs admitted")
        res, surplus = self.keep_picked(admitted, total, pick)
        try:
            await self.confirm(res.placeholders)
        except BaseException:
            await self.release(admitted)
            raise
        return res, surplus

    async def confirm(self, phs: Sequence[Placeholder]) -> None:
        """Clear the candidate mark on the placeholders a pick keeps (one parallel PATCH), so
        they count as the owner's from here on."""
        todo = [p for p in phs if p.candidate]
        if not todo:
            return
        patch = {"metadata": {"annotations": {ANN_CANDIDATE: None}}}
        with trace.span("placement_confirm", placeholders=len(todo)):
            epoch = self.informer.epoch
            res = await asyncio.gather(*[self.kube.patch_pod(p.namespace, p.name, patch)
                                         for p in todo], return_exceptions=True)
        bad = [r for r in res if not isinstance(r, dict)]
        for p, r in zip(todo, res):
            if isinstance(r, dict):
                self.informer.upsert(r, epoch)
                p.candidate = False
        if bad:
            raise ReserveError(f"confirming {len(bad)} placeholder(s) failed: {bad[0]}")

    @staticmethod
    def keep_picked(held: Sequence[Placeholder], total: int,
                    pick: Callable[[List[str]], Sequence[str]]
                    ) -> Tuple[Reservation, List[Placeholder]]:
        """Of admitted placeholders, keep those whose devices ``pick`` chooses (``total`` GPUs;
        a multi-GPU placeholder only as a whole); the rest is surplus."""
        with trace.span("placement_trim"):
            want = set(pick([d for p in held for d in p.device_ids]))
            keep = [p for p in held if p.device_ids and set(p.device_ids) <= want]
            got = sum(len(p.device_ids) for p in keep)
            for p in held:       # pick returned ids we do not hold: fill up with any
                if got >= total:
                    break
                if p not in keep and got + len(p.device_ids) <= total:
                    keep.append(p)
                    got += len(p.device_ids)
        return Reservation(keep), [p for p in held if p not in keep]

    async def _create_claims(self, bodies: List[dict]) -> None:
        """DRA mode: the placeholders' ResourceClaims, before the Pods (a Pod whose claim does
        not exist yet is reported Unschedulable)."""
        claims = [self.claim_for(b) for b in bodies]
        res = await asyncio.gather(*[self.kube.create_claim(c["metadata"]["namespace"], c)
                                     for c in claims], return_exceptions=True)
        errors = [r for r in res if not isinstance(r, dict)]
        if errors:
            await self._delete_claims([(c["metadata"]["namespace"], c["metadata"]["name"])
                                       for c, r in zip(claims, res) if isinstance(r, dict)])
            quota = [e for e in errors if isinstance(e, ApiError) and e.status == 403
                     and "exceeded quota" in _message(e)]
            if quota:   # tenant-namespace claims: the apiserver's quota admission said no
                raise QuotaExceeded(_message(quota[0]))
            raise ReserveError(f"resourceclaim create failed: {errors[0]}")

    async def _delete_claims(self, keys: Sequence[Tuple[str, str]],
                             background: bool = False) -> None:
        if background:
            calls.mark_background()
        res = await asyncio.gather(*[self.kube.delete_claim(ns, n) for ns, n in keys],
                                   return_exceptions=True)
        for (ns, n), r in zip(keys, res):
            if isinstance(r, Exception) and not isinstance(r, NotFound):
                # an unreserved claim holds no device; the reconciler deletes leftovers
                _log.warning("delete resourceclaim %s/%s: %s", ns, n, r)

    async def _delete_unused_claims(self, keys: Sequence[Tuple[str, str]]) -> None:
        """After a failed Pod create: delete the ResourceClaims of the Pods that do not exist.
        A create whose reply was lost may have happened, and a warm-pool placeholder created so
        can already be claimed by an attach: its claim holds that attach's GPU. A claim whose
        Pod could not be read is left to the reconciler, which deletes claims without a Pod."""
        async def absent(ns: str, name: str) -> bool:
            try:
                await self.kube.get_pod(ns, name)
            except NotFound:
                return True
            except Exception:  # noqa: BLE001 - unknown: keep it
                return False
            return False
        gone = await asyncio.gather(*[absent(ns, n) for ns, n in keys])
        await self._delete_claims([k for k, g in zip(keys, gone) if g])

    async def create_pod(self, body: dict, fallback_class: str = "") -> dict:
        """POST one placeholder. If the apiserver refuses its PriorityClass as nonexistent
        (deleted since start, or never applied), the class is recorded as absent and the
        placeholder is created once more with ``fallback_class`` (its tenant's class)."""
        try:
            return await self.kube.create_pod(body["metadata"]["namespace"], body)
        except ApiError as e:
            missing = self._class_missing(e)
            spec = body["spec"]
            if missing is None or spec.get("priorityClassName") != missing:
                raise
            if self.class_values.get(missing, 0) is not None:
                _log.error("PriorityClass %s does not exist: placeholders fall back to their "
                           "tenant's priority (apply deploy/placeholder-priority.yaml)", missing)
            self.class_values[missing] = None
            self.priority_fallbacks += 1
            if fallback_class and fallback_class != missing:
                spec["priorityClassName"] = fallback_class
            else:
                spec.pop("priorityClassName", None)
            return await self.kube.create_pod(body["metadata"]["namespace"], body)

    async def _create(self, bodies: List[dict], owner: Optional[dict] = None
                      ) -> List[Placeholder]:
        fb = ((owner or {}).get("spec") or {}).get("priorityClassName") or ""
        with trace.span("ledger_reserve", placeholders=len(bodies)):
            self.faults.check("ledger_reserve")
            if self.dra:
                await self._create_claims(bodies)
            epoch = self.informer.epoch
            results = await asyncio.gather(*[self.create_pod(b, fb) for b in bodies],
                                           return_exceptions=True)
        created = [Placeholder(r["metadata"]["namespace"], r["metadata"]["name"],
                               r["metadata"]["uid"], (),
                               r["metadata"]["annotations"].get(ANN_MOUNT_MODE, "single"),
                               owner_uid=r["metadata"]["annotations"].get(ANN_OWNER_UID, ""),
                               attach_id=r["metadata"]["annotations"].get(ANN_ATTACH_ID, ""),
                               priority=podu.priority_of(r))
                   for r in results if isinstance(r, dict)]
        for r in results:
            if isinstance(r, dict):
                self.informer.upsert(r, epoch)  # visible to owned_by() before the watch echo
        errors = [r for r in results if not isinstance(r, dict)]
        if errors:
            # a POST that failed may still have created its placeholder (an error after the
            # write, a reply lost after the retries): no watch event need have arrived yet, so
            # neither a follow-up nor a sweep would see it for a while — reap it by its name,
            # which is this attach's alone, before anything else can fail
            await self._reap_unknown([b for b, r in zip(bodies, results)
                                      if not isinstance(r, dict)])
            await self.release(created)
            if self.dra:
                await self._delete_unused_claims(
                    [(b["metadata"]["namespace"], b["metadata"]["name"])
                     for b, r in zip(bodies, results) if not isinstance(r, dict)])
            quota = [e for e in errors if isinstance(e, ApiError) and e.status == 403
                     and "exceeded quota" in _message(e)]
            if quota:   # tenant-namespace placeholders: the apiserver's quota admission said no
                raise QuotaExceeded(_message(quota[0]))
            raise ReserveError(f"placeholder create failed: {errors[0]}")
        try:
            self.faults.check("ledger_reserve", "after")
        except BaseException:
            await self.release(created)
            raise
        return created

    async def _reap_unknown(self, bodies: Sequence[dict]) -> None:
        """Delete whatever exists under the names of ``bodies``, whose create failed: each was
        generated for one attach, so an object of that name with its owner and attach id is a
        create of ours that took effect. The UID comes from a GET (tombstoned first, so the
        DELETED echo is not taken for a foreign delete). What cannot be read or deleted here is
        left to the sweep (a candidate mark or a dead attach gives it away)."""
        for b in bodies:
            md = b["metadata"]
            ann = md.get("annotations") or {}
            try:
                cur = await self.kube.get_pod(md["namespace"], md["name"])
            except NotFound:
                continue                            # the create did not take effect
            except Exception as e:  # noqa: BLE001
                _log.warning("placeholder %s/%s: create failed and the read back failed too: "
                             "%s", md["namespace"], md["name"], e)
                continue
            theirs = cur["metadata"].get("annotations") or {}
            if any(theirs.get(k) != ann.get(k) for k in (ANN_OWNER_UID, ANN_ATTACH_ID)):
                continue
            uid = cur["metadata"].get("uid", "")
            self.tombstones[uid] = asyncio.get_running_loop().time()
            try:
                await self.kube.delete_pod(md["namespace"], md["name"], grace_period_s=0,
                                           uid=uid)
                _log.info("placeholder %s/%s: its create failed but had taken effect; "
                          "deleted", md["namespace"], md["name"])
            except NotFound:
                pass
            except Exception as e:  # noqa: BLE001
                self.tombstones.pop(uid, None)
                _log.warning("placeholder %s/%s: create failed but had taken effect, and the "
                             "delete failed: %s", md["namespace"], md["name"], e)

    async def _await_admission(self, phs: List[Placeholder], timeout: float,
                               tolerant: bool = False) -> List[Placeholder]:
        """Wait until every placeholder is admitted and its devices are in the kubelet ledger.
        ``tolerant``: unschedulable/failed placeholders are returned instead of raising.

        Event-driven: the kubelet ledger is read once per placeholder *event* after binding —
        the bind itself, then the kubelet's first status update, which it posts only after
        admission (device-plugin Allocate) — never in a tight loop: kubelets rate-limit the
        PodResources server (100 qps, burst 10) and reject the excess with RESOURCE_EXHAUSTED.
        Without a new event the ledger is re-read after a backoff of 10 ms doubling to 100 ms.
        The reference instead spins on the apiserver with no sleep until the slave pod is
        Running (reference: pkg/util/gpu/allocator/allocator.go:236-282)."""
        pending = {(p.namespace, p.name): p for p in phs}
        failed: List[Placeholder] = []
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        seen: Dict[Tuple[str, str], str] = {}   # resourceVersion at our last ledger read
        ck = self.checkpoint if self.checkpoint is not None and self.checkpoint.trusted else None
        # DRA: a placeholder's claim allocated and reserved for it (claim watch cache)
        reserved = getattr(self.ledger, "reserved_devices", None) if self.dra else None
        backoff = self.ADMISSION_BACKOFF_CKPT_S if ck is not None else self.ADMISSION_BACKOFF_S
        delay = backoff[0]
        while pending:
            failure: Dict[Tuple[str, str], str] = {}
            from_ckpt: Dict[Tuple[str, str], Tuple[str, ...]] = {}
            bound_keys: List[Tuple[str, str]] = []

            def state():
                fresh = []
                from_ckpt.clear()
                bound_keys.clear()
                for key in pending:
                    pod = self.informer.cache.get(key)
                    # _create put it in the cache, so gone = deleted by someone else (the
                    # reference counted NotFound as success: allocator.go:251-253)
                    if pod is None or pod["metadata"].get("deletionTimestamp"):
                        failure[key] = "placeholder deleted before admission"
                        if not tolerant:
                            return True
                        continue
                    msg = podu.is_unschedulable(pod)
                    if msg and podu.nominated_node(pod):
                        # it preempts lower-priority Pods (a placeholder of a tenant whose own
                        # class preempts) and is bound once they are gone: not a refusal
                        msg = None
                    ids = ck.lookup(pending[key].uid) if ck is not None else None
                    if ids is None and reserved is not None:
                        ids = reserved(key[0], key[1], pending[key].uid)
                    if msg:
                        failure[key] = f"unschedulable: {msg}"
                    elif podu.phase_of(pod) == "Failed":
                        failure[key] = pod["status"].get("reason", "Failed")
                    elif ids:
                        # the kubelet recorded its devices at Allocate (or the scheduler reserved
                        # the DRA claim for it): bound here, whether or not the bind has reached
                        # our watch yet
                        bound_keys.append(key)
                        from_ckpt[key] = ids
                    elif podu.node_of(pod):
                        bound_keys.append(key)
                        news = seen.get(key) != pod["metadata"].get("resourceVersion")
                        if ck is None:
                            if news and (not self.direct or _admitted(pod)):
                                # bound, and news since our last read (bound at creation:
                                # once the kubelet has admitted it)
                                fresh.append(key)
                        else:
                            if news and _admitted(pod):
                                # the kubelet writes the checkpoint at Allocate, before it
                                # posts this status: a miss here means it does not maintain it
                                fresh.append(key)
                    if failure and not tolerant:
                        return True
                return True if failure else (fresh or bool(from_ckpt) or None)

            left = deadline - loop.time()
            if left <= 0:
                raise ReserveError(f"timeout waiting for placeholders {sorted(pending)}")
            try:
                ready = await self.informer.wait_for(
                    state, timeout=min(left, delay) if (seen or (ck and bound_keys)) else left)
            except asyncio.TimeoutError:
                if loop.time() >= deadline:
                    raise ReserveError(f"timeout waiting for placeholders {sorted(pending)}")
                # bound but no news: re-read what is bound, backing off
                ready = [k for k in pending if k in seen or (ck is not None and k in bound_keys)]
                delay = min(delay * 2, backoff[1])
            if failure and not tolerant:
                reason = next(iter(failure.values()))
                if reason.startswith("unschedulable") or reason.startswith("OutOf") or \
                        reason == "UnexpectedAdmissionError":
                    raise InsufficientGPU(reason)
                raise ReserveError(reason)
            for key in failure:
                failed.append(pending.pop(key))
            if from_ckpt:
                self.faults.check("ledger_read")
            for key, ids in list(from_ckpt.items()):    # admitted: known without an RPC
                if key in pending:
                    self._check_count(key, ids)
                    ph = pending.pop(key)
                    ph.device_ids = tuple(ids)
                    self.device_ids[ph.uid] = ph.device_ids
                    self.last_ledger = {**self.last_ledger, key: list(ids)}
                    if ck is not None:
                        self.checkpoint_hits += 1
                        self._checkpoint_misses = 0
            if not pending:
                break
            bound = [k for k in ready if k in pending] if isinstance(ready, list) else []
            if not bound:
                continue
            for k in bound:
                cur = self.informer.cache.get(k)
                seen[k] = cur["metadata"].get("resourceVersion", "") if cur else ""
            # the kubelet records the allocation at admission — read the ledger
            self.faults.check("ledger_read")
            got = None
            if self.cfg.ledger_get and len(bound) <= 4:
                res = await asyncio.gather(*[self.ledger.get(ns, n) for ns, n in bound])
                if all(r is not None for r in res):
                    got = {k: r for k, r in zip(bound, res) if r}
                    merged = dict(self.last_ledger)
                    merged.update(got)
                    self.last_ledger = merged
            if got is None:
                got = await self.ledger.by_pod()
                self.last_ledger = got
            for key in list(pending):
                ids = got.get(key)
                if ids:
                    self._check_count(key, ids)
                    ph = pending.pop(key)
                    ph.device_ids = tuple(ids)
                    self.device_ids[ph.uid] = ph.device_ids
                    if ck is not None and _admitted(self.informer.cache.get(key)) and \
                            ck.lookup(ph.uid) is None:
                        self._checkpoint_misses += 1
                        if self._checkpoint_misses >= self.CHECKPOINT_MISSES:
                            ck.distrust(f"{self._checkpoint_misses} admitted placeholders in "
                                        f"a row had no entry in it")
        return failed

    def _check_count(self, key: Tuple[str, str], ids: Sequence[str]) -> None:
        """The kubelet allocates a placeholder exactly the devices it requests. A ledger that
        reports a different number is inconsistent with the scheduler's accounting (which
        counts the request): mounting those GPUs could double-book one, so the attach fails
        (and is rolled back) instead."""
        pod = self.informer.cache.get(key)
        ann = (pod or {}).get("metadata", {}).get("annotations") or {}
        if not pod:
            want = len(ids)
        elif self.dra or ANN_GPUS in ann:
            want = int(ann.get(ANN_GPUS, len(ids)))
        else:
            want = podu.resource_limit(pod, self.cfg.resource_name)
        if len(ids) != want:
            _log.error("ledger reports %d device(s) %s for placeholder %s/%s, which requests "
                       "%d", len(ids), list(ids), key[0], key[1], want)
            raise ReserveError(f"ledger inconsistent: placeholder {key[1]} requests {want} "
                               f"GPU(s), the kubelet reports {len(ids)}")

    # ------------------------------------------------------------------------ release
    async def _delete(self, p: Placeholder, candidate_only: bool = False) -> Optional[dict]:
        """DELETE one placeholder, only at a version at which it still has the holder the
        caller's view showed (``p.owner_uid``, ``p.attach_id``), so a release decided on a stale
        view never takes a GPU from the Pod that claimed it since (raises :class:`Reowned`).
        Any placeholder can change hands, whatever its name: the surplus of a trim pick goes
        back to the warm pool under its ``<pod>-slave-pod-`` name and is claimed from there.

        ``candidate_only``: released *because* the caller's view shows it an unconfirmed
        candidate of a pick. That view may be a relisted cache from before the pick confirmed
        it (the confirm's write-through is dropped across a relist until a GET re-reads it), and
        a confirmed pick is mounted — so the apiserver's version decides, and the DELETE is
        conditional on it (raises :class:`Reowned` when it is no candidate any more)."""
        if candidate_only:
            return await self._delete_candidate(p)
        if not self.reownable and p.uid:
            # no warm pool: nothing ever claims a placeholder from another holder, so the UID
            # alone pins the object the caller saw. (A version precondition would also trip
            # over the kubelet's status updates, a GET and a second DELETE per detach.)
            return await self.kube.delete_pod(p.namespace, p.name, grace_period_s=0,
                                              uid=p.uid)
        # the cached version only if the cache agrees on the holder; else one read now
        seen = self.informer.cache.get((p.namespace, p.name))
        if seen is None or (p.uid and seen["metadata"].get("uid") != p.uid) or \
                not p.held_by_me(seen):
            seen = await self.kube.get_pod(p.namespace, p.name)
            if p.uid and seen["metadata"].get("uid") != p.uid:
                raise NotFound(404, f"{p.name}: another pod of that name")
            if not p.held_by_me(seen):
                raise Reowned(p.name)
        rv = seen["metadata"].get("resourceVersion", "")
        for attempt in range(self.DELETE_ATTEMPTS):
            try:
                return await self.kube.delete_pod(p.namespace, p.name, grace_period_s=0,
                                                  uid=p.uid or "", resource_version=rv)
            except Conflict:
                # a placeholder being admitted changes with every status the kubelet posts: a
                # conflict with the holder unchanged is that churn, which ends once it runs
                if attempt >= 2:
                    await asyncio.sleep(0.005 * attempt)
                cur = await self.kube.get_pod(p.namespace, p.name)
                if p.uid and cur["metadata"].get("uid") != p.uid:
                    raise NotFound(404, f"{p.name}: another pod of that name") from None
                if not p.held_by_me(cur):
                    raise Reowned(p.name) from None
                rv = cur["metadata"].get("resourceVersion", "")
        raise ApiError(409, f"{p.name} kept changing while being deleted")

    async def _delete_candidate(self, p: Placeholder) -> Optional[dict]:
        for _ in range(self.DELETE_ATTEMPTS):
            cur = await self.kube.get_pod(p.namespace, p.name)
            if p.uid and cur["metadata"].get("uid") != p.uid:
                raise NotFound(404, f"{p.name}: another pod of that name")
            if ANN_CANDIDATE not in (cur["metadata"].get("annotations") or {}) or \
                    not p.held_by_me(cur):
                raise Reowned(p.name)       # confirmed (or claimed) since the caller looked
            try:
                return await self.kube.delete_pod(
                    p.namespace, p.name, grace_period_s=0, uid=p.uid or "",
                    resource_version=cur["metadata"].get("resourceVersion", ""))
            except Conflict:
                continue                    # it changed since the GET: look again
        raise ApiError(409, f"{p.name} kept changing while being deleted")

    async def release(self, phs: Sequence[Placeholder], candidates_only: bool = False) -> None:
        """Delete the placeholders (grace 0, conditional on the holder the caller saw).

        A DELETE answered 200 or 404 ends the release: with grace 0 and no finalizers the
        object is gone from the apiserver, and so from the scheduler's books, when the reply
        comes (the reference's detach also ends at NotFound, allocator.go:284-317). Nothing
        waits for the watch's DELETED echo: the UIDs stay tombstoned until it arrives, so
        every later view (owned_by, live, the free set) already leaves them out. A DELETE whose
        outcome is unknown (5xx, a lost reply, retries exhausted) raises ReserveError and the
        caller's follow-up retries it. ``candidates_only``: each only while the apiserver still
        shows it an unconfirmed candidate of a pick (:meth:`_delete`)."""
        if not phs:
            return
        with trace.span("ledger_release", placeholders=len(phs)):
            self.faults.check("ledger_release")
            # Tombstone before the DELETE is sent: the watch can deliver the DELETED event
            # before the DELETE response, and an un-tombstoned delete reads as a foreign one
            # (→ a spurious revocation and GPURevoked warning on the tenant).
            now = asyncio.get_running_loop().time()
            for p in phs:
                if p.uid:
                    self.tombstones[p.uid] = now
            res = await asyncio.gather(*[self._delete(p, candidates_only) for p in phs],
                                       return_exceptions=True)
            failed, reowned = [], []
            for p, r in zip(phs, res):
                if isinstance(r, Reowned):          # someone else's now: not ours to delete
                    _log.info("placeholder %s/%s changed owner or was confirmed; left to it",
                              p.namespace, p.name)
                    reowned.append(p)
                    if p.uid:
                        self.tombstones.pop(p.uid, None)
                    continue
                if isinstance(r, Exception) and not isinstance(r, NotFound):
                    _log.error("delete placeholder %s/%s: %s", p.namespace, p.name, r)
                    failed.append(p)
                    if p.uid:
                        self.tombstones.pop(p.uid, None)
                else:
                    _log.debug("deleted placeholder %s/%s (owner %s)", p.namespace, p.name,
                               p.owner_uid or "?")
                    # grace 0 + no finalizers: the object is gone from the apiserver (and the
                    # scheduler's books) once DELETE returns; drop it from the cached views
                    if p.uid:
                        cur = self.informer.cache.get((p.namespace, p.name))
                        if cur is None or cur["metadata"].get("uid") != p.uid:
                            self.tombstones.pop(p.uid, None)   # DELETED event already seen
                        self.device_ids.pop(p.uid, None)
                    if isinstance(self.last_ledger, dict):
                        self.last_ledger.pop((p.namespace, p.name), None)
            if self.dra:
                # the claims hold no device once their Pod is gone (deallocated when
                # reservedFor empties); deleting them is cleanup, off the critical path
                gone = [(p.namespace, p.name) for p in phs
                        if p not in failed and p not in reowned]
                if gone:
                    t = asyncio.get_running_loop().create_task(
                        self._delete_claims(gone, background=True))
                    self._bg.add(t)
                    t.add_done_callback(self._bg.discard)
            if failed:
                raise ReserveError(f"could not delete {len(failed)} placeholder(s): "
                                   f"{[p.name for p in failed]}")
            self.faults.check("ledger_release", "after")

    @staticmethod
    def from_pod(p: dict, ledger_ids: Dict[Tuple[str, str], List[str]]) -> Placeholder:
        md = p["metadata"]
        key = (md["namespace"], md["name"])
        ann = md.get("annotations") or {}
        return Placeholder(md["namespace"], md["name"], md.get("uid", ""),
                           tuple(ledger_ids.get(key, ())), ann.get(ANN_MOUNT_MODE, "single"),
                           ANN_CANDIDATE in ann, ann.get(ANN_OWNER_UID) or "",
                           ann.get(ANN_ATTACH_ID) or "", podu.priority_of(p))

    def cached(self, p: dict) -> Optional[Placeholder]:
        """Placeholder with its device IDs from the admission cache (None if unknown)."""
        md = p["metadata"]
        ids = self.device_ids.get(md.get("uid", ""))
        if ids is None:
            return None
        ann = md.get("annotations") or {}
        return Placeholder(md["namespace"], md["name"], md.get("uid", ""), ids,
                           ann.get(ANN_MOUNT_MODE, "single"), ANN_CANDIDATE in ann,
                           ann.get(ANN_OWNER_UID) or "", ann.get(ANN_ATTACH_ID) or "",
                           podu.priority_of(p))
