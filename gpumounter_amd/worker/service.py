"""Worker-side AddGPU / RemoveGPU semantics.

Reference: ``GPUMountImpl.AddGPU`` / ``RemoveGPU`` (reference: pkg/server/gpu-mount/server.go:34-179)
with the policy helpers ``CanMount`` (pkg/util/util.go:207-226), ``GetMountType``
(allocator.go:158-187) and ``GetRemoveGPU`` (allocator.go:101-126). Result enums and their meaning
are identical (see gpumounter_amd/api/gpu_mount.py). Behavioural fixes, each covered by a test:

* per-pod serialization (two concurrent adds on one pod raced in the reference — defect 7);
* ``gpu_num <= 0`` is rejected (reference: division by zero / silent no-op — defect 6);
* mount type comes from the placeholders' recorded mode, not from the "fewer slave pods than
  GPUs" heuristic that misclassifies a pod's own GPUs as an entire mount (defect 5);
* a pod's own device-plugin GPUs are never counted as hot-mounted nor removable (kept from
  allocator.go:112-116), and ``/dev/kfd`` is left alone for such pods;
* the busy check and the kill use one PID snapshot (the reference computed it twice — defect 16);
* every running container is mounted, not just ``ContainerStatuses[0]`` (defect 8);
* a failed mount rolls back cgroup rules and device nodes, not only the slave pods (defect 12).
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import secrets
import time
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import grpc

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.cluster.correction import Correction, ReserveGate, placement_worse
from gpumounter_amd.cluster.informer import PodInformer
from gpumounter_amd.cluster.kube import ApiError, KubeClient, NotFound
from gpumounter_amd.cluster.placeholder import (InsufficientGPU, Placeholder, PlaceholderManager,
                                                ReserveError)
from gpumounter_amd.cluster.quota import GpuQuota, QuotaExceeded
from gpumounter_amd.hw import topology
from gpumounter_amd.hw.inventory import Inventory
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.device import AmdGpu, normalize_device_id
from gpumounter_amd.models.types import (ANN_ATTACH_ID, ANN_IDEMPOTENCY, ANN_MOUNT_MODE,
                                         ANN_OWNER_UID,
                                         ERR_INTERNAL, ERR_POLICY, ERR_QUOTA, LABEL_OWNER_NS,
                                         MODE_DRAINING, MODE_STANDBY, MountType)
from gpumounter_amd.node import procs
from gpumounter_amd.node.hotmount import HotMount, MountError
from gpumounter_amd.node.ledger import LedgerClient, LedgerError
from gpumounter_amd.utils import log, trace
from gpumounter_amd.utils.faults import FaultInjector, InjectedFault
from gpumounter_amd.utils.metrics import Metrics
from gpumounter_amd.worker.drain import DrainKeeper
from gpumounter_amd.worker.lease import LeaseKeeper, expires_of
from gpumounter_amd.worker import planning, status
from gpumounter_amd.worker.notify import Notifier

_log = log.get("worker.service")


class RpcError(Exception):
    def __init__(self, code: grpc.StatusCode, msg: str):
        super().__init__(msg)
        self.code = code
        self.msg = msg


@dataclass
class PodGpuState:
    own: List[AmdGpu] = field(default_factory=list)          # device-plugin GPUs of the pod spec
    hot: List[AmdGpu] = field(default_factory=list)          # hot-mounted via placeholders
    placeholders: List[Placeholder] = field(default_factory=list)
    by_placeholder: Dict[Tuple[str, str], List[AmdGpu]] = field(default_factory=dict)
    mount_type: MountType = MountType.NONE
    ledger: Dict[Tuple[str, str], List[str]] = field(default_factory=dict)  # snapshot used


def can_mount(mount_type: MountType, entire: bool) -> Tuple[bool, str]:
    """Reference util.go:207-226, same decisions, with a reason string."""
    if mount_type == MountType.UNKNOWN:
        return False, "pod mount type is unknown"
    if mount_type != MountType.NONE and entire:
        return False, "pod already has hot-mounted GPUs; entire mount needs an unmounted pod"
    if mount_type == MountType.ENTIRE:
        return False, "pod is entire-mounted; remove its GPUs before adding more"
    return True, ""


class GpuMountService:
    SETTLE_WAIT_S = 2.0          # pod_state: longest wait for the placeholder view to settle
    def __init__(self, cfg, kube: KubeClient, inv: Inventory, ledger: LedgerClient,
                 placeholders: PlaceholderManager, hotmount: HotMount, node_pods: PodInformer,
                 metrics: Optional[Metrics] = None, faults: Optional[FaultInjector] = None) -> None:
        self.cfg = cfg
        self.kube = kube
        self.inv = inv
        self.ledger = ledger
        self.ph = placeholders
        self.hm = hotmount
        self.node_pods = node_pods
        self.metrics = metrics or Metrics()
        self.faults = faults if faults is not None else FaultInjector(cfg.fault)
        self.pool = None  # WarmPool, attached by the Worker when warm_pool_size > 0
        self.plugin = None  # AmdGpuDevicePlugin, attached by the Worker with device_plugin=1
        self.notify = Notifier(cfg, kube)
        self.quota = GpuQuota(cfg, kube)
        self._ns_seen: set = set()
        self.unhealthy: set = set()   # GPU indices failing liveness/ECC (Worker.check_health)
        self.lease = LeaseKeeper(self)
        self.drain = DrainKeeper(self)   # force-removed GPUs whose processes have not exited
        # Reservations that must not interleave on a node run one at a time:
        # * trim briefly holds every free GPU — a concurrent one would see a full node;
        # * device-plugin intents carry no pod identity (GetPreferredAllocation has none), so
        #   two attaches' 1-GPU intents would be indistinguishable to the plugin.
        self._reserve_gate = ReserveGate()
        # a pod's lock lives while a request holds or awaits it: no entry per pod ever seen
        self._locks: "weakref.WeakValueDictionary[Tuple[str, str], asyncio.Lock]" = \
            weakref.WeakValueDictionary()
        self._own: Dict[str, Tuple[str, ...]] = {}   # pod uid → its own device-plugin GPU IDs
        if hasattr(node_pods, "handlers"):
            node_pods.handlers.append(self._forget_pod)
        self.ledger_reads = 0
        self.ledger_reads_checkpoint = 0
        self.adopted = False           # adopt_existing() has run to completion
        # the Reconciler, when the Worker runs one: what a failed operation could not finish (a
        # placeholder release, the rollback to the ledger) is retried with backoff, not left to
        # the periodic sweep (30 s as shipped)
        self.followup = None
        # placeholders of failed attaches whose release is being retried: never replayed as a
        # success under the attach's idempotency key (the client was told it failed). uid →
        # (owner uid, attach id): one that went back to the warm pool and was claimed since is
        # its new holder's, not abandoned
        self.abandoned: Dict[str, Tuple[str, str]] = {}

    # ------------------------------------------------------------------------ helpers
    def pod_lock(self, ns: str, name: str) -> asyncio.Lock:
        lk = self._locks.get((ns, name))
        if lk is None:
            lk = self._locks[(ns, name)] = asyncio.Lock()
        return lk

    def _forget_pod(self, etype: str, pod: dict) -> None:
        """Drop per-pod caches of pods that left the node (a long-lived worker sees many)."""
        if etype == "DELETED":
            self._own.pop(podu.uid_of(pod), None)
            forget = getattr(self.hm.resolver, "forget", None)
            if forget is not None:
                forget(podu.uid_of(pod))
        elif etype == "RELIST":
            live = {podu.uid_of(p) for p in self.node_pods.cache.values()}
            for uid in [u for u in self._own if u not in live]:
                del self._own[uid]

    def is_self(self, pod: dict) -> bool:
        """The worker's own pod (downward API POD_NAME/POD_NAMESPACE): it mounts the host's /dev,
        so nothing may ever be injected into or taken from it."""
        return bool(self.cfg.pod_name) and podu.name_of(pod) == self.cfg.pod_name and \
            podu.ns_of(pod) == (self.cfg.pod_namespace or self.cfg.worker_namespace)

    async def get_pod(self, ns: str, name: str, fresh: bool = False) -> Optional[dict]:
        if not fresh:
            p = self.node_pods.get(ns, name)
            if p is not None and podu.phase_of(p) == "Running":
                return p
        try:
            return await self.kube.get_pod(ns, name)
        except NotFound:
            return None

    def _uid_of(self, key: Tuple[str, str]) -> Optional[str]:
        p = self.node_pods.cache.get(key) or self.ph.informer.cache.get(key)
        return podu.uid_of(p) if p else None

    async def read_ledger(self, authoritative: bool = True, pods: Sequence[dict] = ()
                           ) -> Dict[Tuple[str, str], List[str]]:
        """The node's allocations by (namespace, pod). Non-authoritative reads come from the
        kubelet's device-manager checkpoint when it is in use (no RPC against the rate-limited
        PodResources server); authoritative ones List PodResources and cross-check the
        checkpoint with the answer, so a checkpoint that drifts stops being used."""
        ck = self.ph.checkpoint
        if not authoritative and ck is not None:
            # ``pods``: the ones the caller asks about, which the caches may not hold yet
            led = ck.by_name(list(pods) + list(self.node_pods.cache.values()) +
                             list(self.ph.informer.cache.values()))
            if led is not None:
                self.ledger_reads_checkpoint += 1
                self.ph.last_ledger = led
                return led
        self.ledger_reads += 1
        led = await self.ledger.by_pod()
        self.ph.last_ledger = led
        if ck is not None:
            ck.cross_check(led, self._uid_of)
        return led

    async def pod_state(self, pod: dict, fresh: bool = False,
                        ledger_snapshot: Optional[Dict[Tuple[str, str], List[str]]] = None,
                        authoritative: bool = False) -> PodGpuState:
        """The pod's GPUs from the ledger's point of view.

        Device-plugin allocations never change during a pod's lifetime, so the device IDs of an
        admitted placeholder and a running pod's own GPUs are cached; the kubelet is only asked
        when something is unknown (first sight of a pod, placeholders from a previous worker
        incarnation) or when ``fresh`` is requested (reconciler, status).
        """
        st = PodGpuState()
        # a relist that overtook one of this worker's own writes (a pool claim, a lease) leaves
        # the cache older than what the worker has done until a GET settles it. A view from
        # that cache would, e.g., let a reconcile revoke a just-attached GPU from its Pod, or an
        # attach's complete desired set leave it out: wait for the view to settle
        inf = self.ph.informer
        if not getattr(inf, "settled", True):
            try:
                await inf.wait_for(lambda: inf.settled, self.SETTLE_WAIT_S)
            except asyncio.TimeoutError:
                _log.error("placeholder view not settled %g s after a relist",
                           self.SETTLE_WAIT_S)
                st.mount_type = MountType.UNKNOWN
                return st
        # a failed attach's placeholder that is still being released is nobody's GPU: a rollback
        # or a later attach of the same pod must not mount it (it is schedulable once deleted);
        # nor is a force-removed one whose draining mark is still being retried (worker/drain.py)
        owned = [p for p in self.ph.owned_by(pod)
                 if not self.is_abandoned(p)
                 and p["metadata"].get("uid") not in self.drain.unmarked]
        uid = podu.uid_of(pod)
        cached = [self.ph.cached(p) for p in owned]
        ledger: Optional[Dict[Tuple[str, str], List[str]]] = ledger_snapshot
        if ledger is not None or fresh or uid not in self._own or any(c is None for c in cached):
            try:
                self.faults.check("ledger_read")
                if ledger is None:
                    ledger = await self.read_ledger(authoritative, [pod, *owned])
            except (LedgerError, InjectedFault) as e:
                _log.error("ledger read failed: %s", e)
                st.mount_type = MountType.UNKNOWN
                return st
            self._own[uid] = tuple(ledger.get((podu.ns_of(pod), podu.name_of(pod)), ()))
            phs = [PlaceholderManager.from_pod(p, ledger) for p in owned]
        else:
            phs = cached
        st.ledger = ledger if ledger is not None else self.ph.last_ledger
        keys = self.inv.by_key()

        def resolve(ids) -> List[AmdGpu]:
            out = []
            for d in ids:
                g = keys.get(normalize_device_id(d))
                if g is None:
                    raise LedgerError(f"device id {d!r} from the kubelet ledger is not a GPU of "
                                      f"this node's inventory")
                out.append(g)
            return out

        try:
            st.own = resolve(self._own.get(uid, ()))
            modes = set()
            for ph in phs:
                gs = resolve(ph.device_ids)
                st.placeholders.append(ph)
                st.by_placeholder[(ph.namespace, ph.name)] = gs
                st.hot.extend(gs)
                modes.add(ph.mode)
        except LedgerError as e:
            _log.error("%s", e)
            st.mount_type = MountType.UNKNOWN
            return st
        if not st.placeholders:
            st.mount_type = MountType.NONE
        elif "entire" in modes:
            st.mount_type = MountType.ENTIRE
        else:
            st.mount_type = MountType.SINGLE
        return st

    def prime(self, ledger: Dict[Tuple[str, str], List[str]]) -> int:
        """Seed the per-pod cache of own device-plugin GPUs from the start-up ledger read, for
        every Running pod of the node (their allocation is final once they run): the first
        attach to a pod then needs no PodResources call of its own. Returns how many."""
        n = 0
        for p in self.node_pods.cache.values():
            if podu.phase_of(p) == "Running" and podu.uid_of(p) not in self._own:
                self._own[podu.uid_of(p)] = tuple(ledger.get((podu.ns_of(p), podu.name_of(p)),
                                                             ()))
                n += 1
        return n

    async def warm_up(self) -> None:
        """Run the attach path once before the first request, touching nothing: resolve the
        roctx library, build a placeholder for a synthetic Pod and create it with
        ``dryRun=All`` (the apiserver validates and admits it, stores nothing: the client's
        request path and a keep-alive connection are warm), build and serialize a response
        with devices and stage timings, create the metric children an attach and a detach
        touch. No cgroup, device node or kubelet is involved. (The first attach after a start
        paid for all of it on top of its own work: ``first_attach_ms`` in the bench JSON.)"""
        trace._roctx_lib()                                       # noqa: SLF001
        gpus = self.inv.gpus()[:1]
        fake = {"metadata": {"name": "gm-warm-up", "namespace": "default", "uid": "warm-up"},
                "spec": {"nodeName": self.cfg.node_name, "containers": [{"name": "c"}]},
                "status": {"phase": "Running"}}
        body = self.ph.build(fake, 1, "single", [g.bdf for g in gpus], "add-warm-up", "", "k",
                             1.0)
        try:
            await asyncio.wait_for(self.kube.create_pod(body["metadata"]["namespace"], body,
                                                        dry_run=True), 2.0)
        except Exception as e:  # noqa: BLE001 - an apiserver without dry-run: only a head start
            _log.debug("dry-run placeholder create: %s", e)
        with trace.span("attach") as root:
            with trace.span("ledger_read"):
                st = PodGpuState()
            with trace.span("placement"):
                planning.preferred(self.inv, self.cfg.topology_policy, 1, st,
                                   [g for g in self.inv.gpus() if g.index not in self.unhealthy])
        for cls in (api.AddGPUResponse, api.RemoveGPUResponse):
            r = cls(devices=self._devices(gpus, {}), message="warm-up")
            r.timings.extend(self._timings(root))
            cls.FromString(r.SerializeToString())
        for op in ("add", "remove"):
            for res in ("Success", "INTERNAL"):
                self.metrics.requests.labels(op=op, result=res)
        # the per-stage histograms of the default path: a child is a dozen buckets, and making
        # them on the first attach cost it 0.5 ms on the GPU box (2 ms on a slower host)
        for op, stages in self.WARM_STAGES.items():
            for stage in stages:
                self.metrics.stage_latency.labels(op=op, stage=stage)
        self.metrics.attach_latency.labels(n_gpus="1", mode="single")
        self.metrics.detach_latency.labels(n_gpus="1")

    WARM_STAGES = {"attach": ("pod_lookup", "ledger_read", "placement", "quota",
                              "ledger_reserve", "placeholder_wait", "pool_claim", "mount",
                              "verify"),
                   "detach": ("pod_lookup", "ledger_read", "busy_check", "unmount",
                              "ledger_release", "pool_return")}

    async def reconcile_pod(self, pod: dict,
                            ledger_snapshot: Optional[Dict[Tuple[str, str], List[str]]] = None,
                            authoritative: bool = True) -> List:
        """Make the pod's cgroup rules and /dev nodes equal its (fresh) ledger view.

        Used after any failed attach/detach so a request either fully happens or leaves the pod
        exactly as the ledger describes it, and by the reconciler loop. Returns the issues fixed.
        ``authoritative=False`` (the reconciler, once its sweep has cross-checked the checkpoint
        against PodResources) reads the ledger from the device-manager checkpoint.
        """
        st = await self.pod_state(pod, fresh=True, ledger_snapshot=ledger_snapshot,
                                  authoritative=authoritative)
        if st.mount_type == MountType.UNKNOWN:
            raise LedgerError("ledger unavailable")
        issues = self.hm.audit(pod, st.hot, st.own)
        if not issues:
            return []
        missing = [i for i in issues if i.kind.startswith("missing")]
        stale = [i for i in issues if i.kind.startswith("stale")]
        log.kv(_log, 20, "repairing", pod=f"{podu.ns_of(pod)}/{podu.name_of(pod)}",
               hot=[g.bdf for g in st.hot], placeholders=[ph.name for ph in st.placeholders],
               issues=sorted({f"{i.kind} {i.path}" for i in issues}))
        if missing:
            self.hm.repair(pod, missing, st.hot, st.own)
        if stale:
            self.hm.revoke_issues(pod, stale, st.hot, st.own)
        return issues

    async def adopt_existing(self) -> int:
        """Seed the injection journal from the ledger for every live owner that has
        hot-mounted GPUs but no journal record (node/hotmount.py ``adopt``): the upgrade path
        from a worker without a journal, or one whose state_dir was lost. Runs once, before the
        worker serves, and again from the reconciler until it has succeeded."""
        if self.adopted:
            return 0
        owners: Dict[Tuple[str, str], str] = {}
        for p in self.ph.live():
            md = p["metadata"]
            ann = md.get("annotations") or {}
            if ann.get(ANN_MOUNT_MODE) in (MODE_STANDBY, MODE_DRAINING):
                continue
            ons = (md.get("labels") or {}).get(LABEL_OWNER_NS, "")
            oname = ann.get("gpumounter.amd.com/owner-name", "")
            if oname:
                owners[(ons, oname)] = ann.get(ANN_OWNER_UID, "")
        n = 0
        for (ns, name), uid in owners.items():
            pod = self.node_pods.get(ns, name)
            if pod is None or podu.uid_of(pod) != uid or podu.phase_of(pod) != "Running" or \
                    self.is_self(pod):
                continue
            async with self.pod_lock(ns, name):
                st = await self.pod_state(pod, ledger_snapshot=self.ph.last_ledger or None)
                if st.mount_type == MountType.UNKNOWN:
                    return n                     # ledger unreadable: the reconciler retries
                try:
                    n += self.hm.adopt(pod, st.hot, st.own)
                except Exception as e:  # noqa: BLE001 - a container that went away meanwhile
                    _log.warning("journal adoption for %s/%s: %s", ns, name, e)
        self.adopted = True
        if n:
            log.kv(_log, 30, "adopted hot-mount state with no journal record", entries=n,
                   owners=len(owners))
        return n

    def _current(self, pod: dict) -> dict:
        """The pod as the node informer holds it now (same UID): a container restart seen
        while this request waited for the pod's lock must not send it to the old container."""
        cur = self.node_pods.get(podu.ns_of(pod), podu.name_of(pod))
        return cur if cur is not None and podu.uid_of(cur) == podu.uid_of(pod) else pod

    async def _rollback(self, pod: dict, what: str) -> bool:
        """Reconcile the pod to its ledger state after a failed operation. Returns True if the
        pod itself is gone (deleted or replaced meanwhile): nothing is left to repair then."""
        try:
            cur = await self.get_pod(podu.ns_of(pod), podu.name_of(pod), fresh=True)
            if cur is None or podu.uid_of(cur) != podu.uid_of(pod) or \
                    podu.phase_of(cur) != "Running":
                log.kv(_log, 20, f"{what} rollback: pod is gone, nothing left on the node",
                       pod=f"{podu.ns_of(pod)}/{podu.name_of(pod)}")
                return True
            fixed = await self.reconcile_pod(cur)
            if fixed:
                log.kv(_log, 30, f"{what} rolled back to ledger state",
                       pod=f"{podu.ns_of(pod)}/{podu.name_of(pod)}", fixed=len(fixed))
        except Exception as e:  # noqa: BLE001
            _log.error("rollback after %s failed (retried by the reconciler): %s", what, e)
            self._follow_up(pod)
        return False

    def is_abandoned(self, p: dict) -> bool:
        """``p`` is a failed attach's placeholder, still held by that attach."""
        held = self.abandoned.get(p["metadata"].get("uid", ""))
        if held is None:
            return False
        ann = p["metadata"].get("annotations") or {}
        return (ann.get(ANN_OWNER_UID) or "") == held[0] and \
            (not held[1] or (ann.get(ANN_ATTACH_ID) or "") == held[1])

    def _follow_up(self, pod: dict, drop: Sequence[Placeholder] = ()) -> None:
        """Hand what this operation could not finish to the reconciler's retrying follow-up:
        release ``drop`` (placeholders of a failed attach) and reconcile the pod to its ledger."""
        self.abandoned.update({p.uid: (p.owner_uid, p.attach_id) for p in drop if p.uid})
        if self.followup is not None:
            self.followup(podu.ns_of(pod), podu.name_of(pod), drop)

    async def _release_or_follow_up(self, pod: dict, phs: Sequence[Placeholder],
                                    what: str) -> None:
        """Release a failed attach's placeholders; one that cannot be deleted now is retried by
        the reconciler until it is (its GPU is nobody's: the client was told the attach failed)."""
        try:
            await self._release(phs)
        except Exception as e:  # noqa: BLE001
            _log.error("placeholder release after %s: %s", what, e)
            self._follow_up(pod, phs)

    @staticmethod
    def _devices(gs: Sequence[AmdGpu], owner: Dict[int, str]) -> List:
        return [api.Device(uuid=g.uuid, bdf=g.bdf, index=g.index, render_minor=g.render_minor,
                           card_minor=g.card_minor, numa_node=g.numa_node,
                           xgmi_hive_id=g.xgmi_hive_id, placeholder=owner.get(g.index, ""))
                for g in gs]

    SLOW_ATTACH_MS = 50.0
    # a deleted Pod's devices are freed by the kubelet once it has stopped the Pod (tens to
    # hundreds of ms after the DELETE's answer): until then it refuses a placeholder that needs
    # them at admission (UnexpectedAdmissionError, or OutOf<resource> for a directly bound one)
    # although the scheduler, and our own ledger view, count them free — after a detach or a
    # yield of standbys. Such a refusal is retried after these delays, each time with a new
    # placeholder (whose own scheduling and admission take time too, so the first retry goes
    # at once); a refusal with no GPU free in our view is answered at once
    ADMISSION_RETRY_S = (0.0, 0.01, 0.02, 0.04, 0.08, 0.16, 0.32)
    LEASE_REBASE_S = 1.0     # an attach slower than this re-stamps its lease (_lease_booked)

    def _count_error(self, op: str, e: BaseException) -> None:
        """RPCs that end in a gRPC error count under its status name (RESOURCE_EXHAUSTED = quota,
        FAILED_PRECONDITION = mount-type refusal, INTERNAL = a failed and rolled-back operation)."""
        code = e.code.name if isinstance(e, RpcError) else "INTERNAL"
        self.metrics.requests.labels(op=op, result=code).inc()

    @staticmethod
    def _timings(root: trace.Span) -> List:
        return [api.StageTiming(name=k, ms=v) for k, v in root.flat().items()]

    # ------------------------------------------------------------------------ AddGPU
    async def add_gpu(self, req) -> "api.AddGPUResponse":
        rid = req.request_id or log.new_request_id("add")
        with self.notify.operation(), log.with_rid(rid), \
                trace.span("attach", pod=f"{req.namespace}/{req.pod_name}",
                           n=req.gpu_num, entire=req.is_entire_mount) as root:
            try:
                resp = await self._add_gpu(req)
            except Exception as e:
                self._count_error("add", e)
                raise
        resp.total_ms = root.duration_ms
        resp.timings.extend(self._timings(root))
        if root.duration_ms > self.SLOW_ATTACH_MS:
            # the stage split of a slow attach, for tail-latency attribution from the logs
            _log.warning("slow attach %s/%s: %.1f ms %s", req.namespace, req.pod_name,
                         root.duration_ms, {k: round(v, 2) for k, v in root.flat().items()})
        result = api.AddGPUResponse.AddGPUResult.Name(resp.add_gpu_result)
        self.metrics.requests.labels(op="add", result=result).inc()
        if resp.add_gpu_result == api.ADD_SUCCESS:
            self.metrics.attach_latency.labels(
                n_gpus=str(req.gpu_num), mode="entire" if req.is_entire_mount else "single"
            ).observe(root.duration_ms / 1e3)
            self.metrics.observe_trace("attach", root)
        return resp

    @staticmethod
    def _check_names(req) -> None:
        bad = podu.name_error(req.namespace, req.pod_name)
        if bad is not None:
            raise RpcError(grpc.StatusCode.INVALID_ARGUMENT, bad)

    async def _add_gpu(self, req):
        self._check_names(req)
        n = int(req.gpu_num)
        if n <= 0 or n > self.cfg.max_gpus_per_request:
            raise RpcError(grpc.StatusCode.INVALID_ARGUMENT, f"invalid gpu_num {n}")
        with trace.span("pod_lookup"):
            self.faults.check("pod_lookup")
            pod = await self.get_pod(req.namespace, req.pod_name)
        if pod is None:
            _log.info("no such pod %s/%s", req.namespace, req.pod_name)
            return api.AddGPUResponse(add_gpu_result=api.ADD_POD_NOT_FOUND)
        if self.cfg.node_name and podu.node_of(pod) != self.cfg.node_name:
            raise RpcError(grpc.StatusCode.FAILED_PRECONDITION,
                           f"pod is on node {podu.node_of(pod)!r}, this worker serves "
                           f"{self.cfg.node_name!r}")
        if self.is_self(pod):
            raise RpcError(grpc.StatusCode.FAILED_PRECONDITION,
                           f"{ERR_POLICY}: the gpumounter worker pod itself is never a target")
        async with self.pod_lock(req.namespace, req.pod_name):
            pod = self._current(pod)
            if podu.phase_of(pod) != "Running":
                pod = await self.get_pod(req.namespace, req.pod_name, fresh=True)
                if pod is None:
                    return api.AddGPUResponse(add_gpu_result=api.ADD_POD_NOT_FOUND)
                if podu.phase_of(pod) != "Running":
                    raise RpcError(grpc.StatusCode.FAILED_PRECONDITION,
                                   f"pod phase is {podu.phase_of(pod)}, not Running")
            with trace.span("ledger_read"):
                st = await self.pod_state(pod)
            if req.idempotency_key:
                replay = await self._replay(pod, st, req.idempotency_key, req.lease_s)
                if replay is not None:
                    return replay
            ok, why = can_mount(st.mount_type, req.is_entire_mount)
            if not ok:
                _log.warning("policy denied add on %s/%s: %s", req.namespace, req.pod_name, why)
                raise RpcError(grpc.StatusCode.FAILED_PRECONDITION, f"{ERR_POLICY}: {why}")
            with trace.span("placement"):
                free = self._free(st)
                preferred = self._preferred(n, st, free)
            # a lease is part of the booking: every placeholder is created (or claimed) with it,
            # so no crash can leave a leased GPU booked without one
            lease_exp = time.time() + req.lease_s if req.lease_s > 0 else 0.0
            try:
                async with self._quota_guard(req.namespace, n):
                    res = await self._reserve(pod, n, req, st, preferred, len(free), lease_exp)
                    await self._quota_recheck(req.namespace, n, res)
            except QuotaExceeded as e:
                _log.info("quota refused %d GPU(s) for %s/%s: %s", n, req.namespace,
                          req.pod_name, e)
                self.notify.event(pod, "GPUAttachFailed", str(e), warning=True)
                raise RpcError(grpc.StatusCode.RESOURCE_EXHAUSTED, f"{ERR_QUOTA}: {e}") from e
            except InsufficientGPU as e:
                _log.info("insufficient GPUs on %s: %s", self.cfg.node_name, e)
                self.notify.event(pod, "GPUAttachFailed",
                                  f"{n} GPU(s) requested, node {self.cfg.node_name} cannot "
                                  f"provide them: {e}", warning=True)
                return api.AddGPUResponse(add_gpu_result=api.ADD_INSUFFICIENT, message=str(e))
            except (ReserveError, asyncio.TimeoutError, InjectedFault, LedgerError) as e:
                # a reservation that failed part-way may leave placeholders its own cleanup
                # could not delete (candidates of a trim/correction pick among them): the
                # follow-up releases what no attach holds any more, without waiting for a sweep
                self._follow_up(pod)
                raise RpcError(grpc.StatusCode.INTERNAL, f"{ERR_INTERNAL}: {e}") from e
            keys = self.inv.by_key()
            new = [keys[normalize_device_id(d)] for d in res.device_ids]
            owner = {}
            for ph in res.placeholders:
                for d in ph.device_ids:
                    owner[keys[normalize_device_id(d)].index] = ph.name
            want = res.preferred or preferred
            if want and sorted(normalize_device_id(d) for d in res.device_ids) != \
                    sorted(normalize_device_id(d) for d in want):
                self.metrics.placement_mismatch.inc()
            try:
                pod = self._current(pod)         # a restart seen while reserving
                with trace.span("mount", gpus=len(new)):
                    targets = self.hm.attach(pod, new, st.hot, st.own, req.container)
                if self.cfg.attach_verify:
                    with trace.span("verify"):
                        self.faults.check("verify")
                        issues = self.hm.verify(pod, list(st.hot) + new, st.own,
                                                req.container, targets)
                    if issues:
                        self.metrics.verify_failures.inc()
                        raise MountError("attach did not take effect: " + ", ".join(
                            f"{i.container}:{i.kind}:{i.path}" for i in issues[:4]))
            except (MountError, InjectedFault) as e:
                _log.error("mount failed on %s/%s: %s", req.namespace, req.pod_name, e)
                await self._release_or_follow_up(pod, res.placeholders, "a failed mount")
                if await self._rollback(pod, "attach"):   # deleted while we were attaching
                    return api.AddGPUResponse(add_gpu_result=api.ADD_POD_NOT_FOUND,
                                              message=f"pod went away during the attach: {e}")
                raise RpcError(grpc.StatusCode.INTERNAL, f"{ERR_INTERNAL}: {e}") from e
            if self._owner_gone(pod):
                # deleted (maybe re-created under its name) while the attach ran, before the
                # placeholders existed: the DELETED event's release found nothing to release
                _log.warning("pod %s/%s was deleted during the attach; releasing its GPUs",
                             req.namespace, req.pod_name)
                await self._release_or_follow_up(pod, res.placeholders, "an attach into a "
                                                                         "deleted pod")
                return api.AddGPUResponse(add_gpu_result=api.ADD_POD_NOT_FOUND,
                                          message="pod went away during the attach")
            msg = "Add GPU Success"
            if lease_exp:
                lease_exp = await self._lease_booked(pod, res.placeholders, lease_exp,
                                                     req.lease_s)
                msg += time.strftime(" (lease until %Y-%m-%dT%H:%M:%SZ)", time.gmtime(lease_exp))
            log.kv(_log, 20, "attached", pod=f"{req.namespace}/{req.pod_name}",
                   gpus=[g.bdf for g in new], by=req.requested_by, lease_s=req.lease_s)
            self.notify.attached(pod, new, list(st.hot) + new,
                                 "entire" if req.is_entire_mount else "single",
                                 by=req.requested_by)
            return api.AddGPUResponse(add_gpu_result=api.ADD_SUCCESS,
                                      devices=self._devices(new, owner), message=msg)

    async def _lease_booked(self, pod: dict, phs, lease_exp: float, lease_s: float) -> float:
        """Arm the lease the placeholders were booked with. The booking stamped it when the
        request arrived, so an attach that waited long for admission (a slow scheduler, up to
        ``attach_timeout_s``) would have spent part of the lease before the tenant got the GPU
        — all of it, for a lease shorter than the wait. Past ``LEASE_REBASE_S`` the lease is
        re-stamped from now (one PATCH per placeholder); the booking carried a lease from the
        start either way, so no crash leaves a leased GPU without one."""
        if time.time() - (lease_exp - lease_s) <= self.LEASE_REBASE_S:
            self.lease.booked(pod, phs, lease_exp)      # timers; no write
            return lease_exp
        try:
            return await self.lease.grant(pod, phs, lease_s)
        except Exception as e:  # noqa: BLE001 - the booked lease still holds
            _log.warning("re-stamping the lease of %s/%s after a slow attach: %s",
                         podu.ns_of(pod), podu.name_of(pod), e)
            self.lease.booked(pod, phs, lease_exp)
            return lease_exp

    @contextlib.asynccontextmanager
    async def _quota_guard(self, ns: str, n: int):
        """Quota check before reserving; same-namespace attaches on this node serialise on it."""
        if not self.quota.active:
            yield
            return
        async with self.quota.lock(ns):
            with trace.span("quota"):
                try:
                    await self.quota.check(ns, n)
                except ApiError as e:
                    raise RpcError(grpc.StatusCode.INTERNAL,
                                   f"{ERR_INTERNAL}: quota lookup: {e}") from e
            yield

    async def _quota_recheck(self, ns: str, n: int, res) -> None:
        if not self.quota.active or not (await self.quota.limits(ns)):
            return
        try:
            await self.quota.recheck(ns, n)
        except QuotaExceeded:
            await self._release(res.placeholders)
            raise

    async def _replay(self, pod: dict, st: PodGpuState, key: str, lease_s: float = 0.0):
        """A retried request (same idempotency key) returns the earlier attach instead of adding
        more GPUs; the mount itself is re-checked (repair) so a half-finished attempt completes,
        and so is its lease: an attempt cut off (worker killed) between the mount and the lease
        annotation would otherwise hand back GPUs that never expire."""
        raw = {p["metadata"]["name"]: p for p in self.ph.owned_by(pod)
               if (p["metadata"].get("annotations") or {}).get(ANN_IDEMPOTENCY) == key
               and not self.is_abandoned(p)
               and p["metadata"].get("uid") not in self.drain.unmarked}
        mine = set(raw)
        if not mine:
            return None
        if lease_s > 0:
            unleased = [ph for ph in st.placeholders if ph.name in mine and
                        expires_of(raw[ph.name]) is None and
                        self.lease.granted(raw[ph.name]) is None]
            if unleased:
                await self.lease.grant(pod, unleased, lease_s)
        gs, owner = [], {}
        for ph in st.placeholders:
            if ph.name in mine:
                for g in st.by_placeholder[(ph.namespace, ph.name)]:
                    gs.append(g)
                    owner[g.index] = ph.name
        issues = self.hm.audit(pod, st.hot, st.own)
        missing = [i for i in issues if i.kind.startswith("missing")]
        if missing:
            self.hm.repair(pod, missing, st.hot, st.own)
        log.kv(_log, 20, "idempotent replay", key=key, gpus=[g.bdf for g in gs])
        return api.AddGPUResponse(add_gpu_result=api.ADD_SUCCESS,
                                  devices=self._devices(gs, owner),
                                  message="Add GPU Success (replayed)")

    async def _reserve(self, pod: dict, n: int, req, st: PodGpuState, preferred: List[str],
                       n_free: int = 0, lease_exp: float = 0.0):
        """Claim from the warm pool first (if enabled), create placeholders for the rest.

        Placement (``placement_enforce``): the device plugin decides which GPUs a placeholder
        gets, and a stock plugin never sees gpumounter's preferred set. ``auto`` (default)
        checks what was admitted against the best set and, when it is worse, corrects it by
        holding the node's other free GPUs and keeping the best ones (:meth:`_correct`); an
        exact path is used instead when one exists — gpumounter's own device plugin (intents
        answered by GetPreferredAllocation) or a DRA claim pinned by a CEL selector. ``trim``
        always holds every free GPU; ``hint`` only annotates the preferred set."""
        pool = self.pool if self.pool is not None and self.pool.enabled else None
        planned = {p.uid for p in pool.standby()} if pool is not None else set()
        refused = pool.refusals if pool is not None else 0
        try:
            return await self._reserve_once(pod, n, req, st, preferred, n_free, lease_exp)
        except InsufficientGPU:
            # a refill that started before this attach held GPUs this attach's plan took for
            # free (its standby placeholders were not admitted yet): claim those instead — or,
            # when the kubelet refused the refill (a teardown in flight) and it gave them up,
            # book them again
            if pool is None or not await pool.admitted(self.cfg.attach_timeout_s):
                raise
            if not {p.uid for p in pool.standby()} - planned and pool.refusals == refused:
                raise
            _log.info("attach refused while the pool refilled; booking again")
            return await self._reserve_once(pod, n, req, st, preferred, n_free, lease_exp)

    async def _reserve_once(self, pod: dict, n: int, req, st: PodGpuState,
                            preferred: List[str], n_free: int = 0, lease_exp: float = 0.0):
        dra = self.cfg.gpu_allocation == "dra"     # the claim's selector pins the devices
        mode = self.cfg.placement_enforce
        if (mode != "trim" or dra) and self.plugin is None:
            async with self._reserve_gate.shared():
                res = await self._reserve_unlocked(pod, n, req, st, preferred, n_free, lease_exp)
            if mode == "auto" and not dra and res.corrigible and \
                    self._placement_worse(st, res.device_ids, preferred):
                async with self._reserve_gate.exclusive():
                    res = await self._correct(pod, n, req, st, res, lease_exp)
            return res
        async with self._reserve_gate.exclusive():
            # recompute against the ledger as it is now that we hold the node
            free = self._free(st)
            preferred = self._preferred(n, st, free)
            res = await self._reserve_unlocked(pod, n, req, st, preferred, len(free), lease_exp)
            if not res.preferred:
                res.preferred = list(preferred)
            return res

    def _placement_worse(self, st: PodGpuState, got: Sequence[str],
                         want: Sequence[str]) -> bool:
        return placement_worse(self.inv, st.hot + st.own, got, want,
                               getattr(self.cfg, "placement_correct_on", "numa"))

    async def _correct(self, pod: dict, n: int, req, st: PodGpuState, res,
                       lease_exp: float = 0.0):
        """Swap the plugin's worse-placed choice for the best free set (cluster/correction.py:
        hold every other free GPU, keep the best ``n``, release the rest)."""
        c = Correction(self.ph, self.inv, self._free(st), st.hot + st.own, pod, n,
                       req.is_entire_mount, secrets.token_hex(4) if req.is_entire_mount else "",
                       log.request_id.get(), req.container, req.idempotency_key,
                       self.cfg.topology_policy, self.faults,
                       lambda phs: self._release_quiet(pod, phs), lease_exp)
        try:
            out = await c.run(res)
        finally:
            if c.error is not None:
                # a hold that failed part-way may have left candidates no book of the
                # correction holds: the follow-up finds them by their mark, now rather than at
                # the next periodic sweep
                self._follow_up(pod)
        if c.corrected:
            self.metrics.placement_corrections.inc()
        return out

    async def _release_quiet(self, pod: dict, phs) -> None:
        try:
            await self._release([p for p in phs if p.device_ids]
                                + [p for p in phs if not p.device_ids])
        except Exception as e:  # noqa: BLE001 - the reconciler's follow-up retries
            _log.error("releasing placeholders: %s", e)
            self._follow_up(pod, phs)

    async def _reserve_unlocked(self, pod: dict, n: int, req, st: PodGpuState,
                                preferred: List[str], n_free: int, lease_exp: float = 0.0):
        claimed = None
        create_pref = preferred
        # standbys this Pod may claim: those that rank at least as high as a placeholder of
        # its own would (cluster/placeholder.py priority_for; priority is immutable)
        rank = self.ph.priority_for(pod)[1]
        pool_on = self.pool is not None and self.pool.enabled
        if pool_on and self.pool.standby(rank):
            plan = self._plan_with_pool(n, st, rank)
            if plan is not None and plan[0]:
                claim_idx, plan_pref = plan
                claimed = await self.pool.claim(pod, len(claim_idx), req.is_entire_mount,
                                                st.hot + st.own, log.request_id.get(),
                                                req.container, req.idempotency_key,
                                                want=claim_idx, lease_expires=lease_exp,
                                                min_priority=rank)
                if claimed is not None:
                    create_pref = plan_pref
        got = len(claimed.placeholders) if claimed else 0
        if got == n:
            claimed.preferred = claimed.device_ids       # claimed by exact device
            return claimed
        if got:
            preferred = create_pref
        if not got and preferred and self.cfg.placement_enforce == "trim" and n_free > n \
                and self.cfg.gpu_allocation != "dra":
            try:
                return await self._reserve_trim(pod, n, req, st, n_free, lease_exp)
            except QuotaExceeded as e:
                # tenant-namespace placeholders: holding every free GPU can exceed the
                # tenant's quota although the request fits; reserve it plainly instead
                _log.info("trim refused by the tenant's quota (%s); plain reservation", e)
        yielded = []
        if pool_on and n - got > 0:
            if self.pool.refilling():
                # low standbys being admitted would take GPUs that look free here
                await self.pool.cancel_pending_low(rank)
            free_now = self._free(st)
            if len(free_now) < n - got:
                # the rest is held by standbys that rank below this Pod: give them back to the
                # scheduler and book their GPUs at this Pod's rank instead
                yielded = await self.pool.yield_low(n - got - len(free_now), rank,
                                                    st.hot + st.own)
                if yielded:
                    keys = self.inv.by_key()
                    back = [keys[normalize_device_id(ph.device_ids[0])] for ph in yielded
                            if normalize_device_id(ph.device_ids[0]) in keys]
                    preferred = planning.preferred(self.inv, self.cfg.topology_policy, n - got,
                                                   st, free_now + back)
        token = ""
        if self.plugin is not None and preferred:
            # our own device plugin answers GetPreferredAllocation for these placeholders
            token = log.request_id.get() or secrets.token_hex(4)
            for ids in ([preferred] if req.is_entire_mount else [[d] for d in preferred]):
                self.plugin.intend(ids, token)
        try:
            delays = list(self.ADMISSION_RETRY_S)
            while True:
                try:
                    rest = await self.ph.reserve(pod, n - got, req.is_entire_mount, preferred,
                                                 attach_id=log.request_id.get(),
                                                 container=req.container,
                                                 idempotency_key=req.idempotency_key,
                                                 lease_expires=lease_exp)
                    break
                except InsufficientGPU as e:
                    kubelet = str(e).startswith(("UnexpectedAdmissionError", "OutOf"))
                    transient = yielded or (kubelet and self._room(st) >= n - got)
                    if not delays or not transient:
                        if kubelet:
                            # "full": no room in our view either (the kubelet's refusal of a
                            # directly bound placeholder on a full node); "exhausted": the GPUs
                            # looked free the whole time, and the kubelet kept refusing
                            self.metrics.admission_refusals.labels(
                                outcome="exhausted" if transient else "full").inc()
                        raise
                    self.metrics.admission_refusals.labels(outcome="rebooked").inc()
                    # a kubelet that has not torn a deleted Pod down yet refuses its devices
                    # at admission: again, a moment later
                    _log.info("placeholder refused at admission (%s) with GPUs free in the "
                              "ledger; retrying in %g s", e, delays[0])
                    delay = delays.pop(0)
                    if delay:
                        await asyncio.sleep(delay)
        except BaseException:
            if claimed:
                await self.pool.give_back(claimed.placeholders)
            raise
        finally:
            if token:
                self.plugin.withdraw(token)
        if claimed:
            rest.placeholders = claimed.placeholders + rest.placeholders
            rest.preferred = claimed.device_ids + list(preferred) if preferred else []
        else:
            rest.preferred = list(preferred)
            # a plain reservation of the plugin's choosing, with other free GPUs to choose from
            rest.corrigible = not token and len(preferred) == n and n_free > n
        return rest

    async def _release(self, phs) -> None:
        if self.pool is not None and self.pool.enabled:
            await self.pool.give_back(phs)
        else:
            await self.ph.release(phs)

    def _plan_with_pool(self, n: int, st: PodGpuState, rank: Optional[int] = None):
        return planning.plan_with_pool(self.inv, self.cfg.topology_policy,
                                       self.pool.standby(rank), n, st, self._free(st))

    async def _reserve_trim(self, pod: dict, n: int, req, st: PodGpuState, width: int,
                            lease_exp: float = 0.0):
        keys = self.inv.by_key()
        attached = st.hot + st.own

        def pick(ids: List[str]) -> List[str]:
            held = {keys[normalize_device_id(d)].index: d for d in ids
                    if normalize_device_id(d) in keys}
            plc = topology.choose([keys[normalize_device_id(d)] for d in held.values()], n,
                                  self.inv.links(), attached=attached,
                                  policy=self.cfg.topology_policy)
            return [held[i] for i in plc.chosen] if plc else []

        res, surplus = await self.ph.reserve_trim(
            pod, n, req.is_entire_mount, width, pick, attach_id=log.request_id.get(),
            container=req.container, idempotency_key=req.idempotency_key,
            lease_expires=lease_exp)
        res.preferred = res.device_ids                    # trim keeps exactly what it picked
        if surplus:
            with trace.span("placement_release", placeholders=len(surplus)):
                await self._release_quiet(pod, surplus)
        return res

    def _free(self, st: PodGpuState) -> List[AmdGpu]:
        return planning.free_gpus(self.inv, self.ph, self.unhealthy, st)

    def _owner_gone(self, pod: dict) -> bool:
        """The node-pod watch has seen ``pod`` (this UID) deleted, or its name taken by a new
        Pod."""
        key, uid = (podu.ns_of(pod), podu.name_of(pod)), podu.uid_of(pod)
        if getattr(self.node_pods, "deleted", {}).get(key) == uid:
            return True
        cur = self.node_pods.cache.get(key)
        return cur is not None and podu.uid_of(cur) != uid

    def _room(self, st: PodGpuState) -> int:
        """GPUs free once the kubelet has torn down the Pods gone from the apiserver: those no
        live Pod holds in the ledger view (which can still list deleted Pods, or be older than
        the teardown) nor a placeholder of ours."""
        held = {normalize_device_id(d) for uid, ids in self.ph.device_ids.items()
                if uid not in self.ph.tombstones for d in ids}
        for (ns, name), ids in st.ledger.items():
            p = self.node_pods.get(ns, name) or self.ph.informer.cache.get((ns, name))
            if p is not None and p["metadata"].get("uid") not in self.ph.tombstones and \
                    not p["metadata"].get("deletionTimestamp"):
                held.update(normalize_device_id(d) for d in ids)
        return sum(1 for g in self.inv.gpus()
                   if not held.intersection(g.ledger_keys()) and g.index not in self.unhealthy)

    def _preferred(self, n: int, st: PodGpuState, free: Optional[List[AmdGpu]] = None
                   ) -> List[str]:
        return planning.preferred(self.inv, self.cfg.topology_policy, n, st,
                                  self._free(st) if free is None else free)

    # ------------------------------------------------------------------------ RemoveGPU
    async def remove_gpu(self, req) -> "api.RemoveGPUResponse":
        rid = req.request_id or log.new_request_id("rm")
        with self.notify.operation(), log.with_rid(rid), \
                trace.span("detach", pod=f"{req.namespace}/{req.pod_name}",
                           n=len(req.uuids), force=req.force) as root:
            try:
                resp = await self._remove_gpu(req)
            except Exception as e:
                self._count_error("remove", e)
                raise
        resp.total_ms = root.duration_ms
        resp.timings.extend(self._timings(root))
        result = api.RemoveGPUResponse.RemoveGPUResult.Name(resp.remove_gpu_result)
        self.metrics.requests.labels(op="remove", result=result).inc()
        if resp.remove_gpu_result == api.REMOVE_SUCCESS:
            self.metrics.detach_latency.labels(n_gpus=str(len(req.uuids))).observe(
                root.duration_ms / 1e3)
            self.metrics.observe_trace("detach", root)
        return resp

    async def _remove_gpu(self, req):
        self._check_names(req)
        with trace.span("pod_lookup"):
            self.faults.check("pod_lookup")
            pod = await self.get_pod(req.namespace, req.pod_name)
        if pod is None:
            return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_POD_NOT_FOUND)
        async with self.pod_lock(req.namespace, req.pod_name):
            pod = self._current(pod)
            with trace.span("ledger_read"):
                st = await self.pod_state(pod)
            if st.mount_type == MountType.UNKNOWN:
                raise RpcError(grpc.StatusCode.INTERNAL, f"{ERR_INTERNAL}: ledger unavailable")
            selected = self.select_removal(st, list(req.uuids))
            if not selected:
                return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_GPU_NOT_FOUND,
                                             message="Invalid UUIDs")
            sel_idx = {g.index for g in selected}
            keep = [g for g in st.hot if g.index not in sel_idx]
            pinned: Optional[procs.Pinned] = None
            try:
                with trace.span("busy_check"):
                    self.faults.check("busy_check")
                    targets = self.hm.resolve(pod, req.container)
                    # privileged containers get no rule/node writes, but their processes use
                    # the GPU all the same: they count for busy and are killed by force
                    everyone = self.hm.resolve(pod, req.container, include_privileged=True) \
                        if any(r.privileged for r in podu.running_containers(pod, req.container)) \
                        else targets
                    cpids = sorted({p for t in everyone for p in t.pids})
                    # pin the snapshot, then confirm membership: from here on a recycled PID
                    # cannot be mistaken for a container process (node/procs.py Pinned)
                    pinned = procs.Pinned(cpids)
                    if pinned.fds:
                        pinned.restrict({p for t in everyone
                                         for p in self.hm.resolver.pids(t.cgdir)})
                    real = not self.inv.is_mock
                    busy = procs.busy_pids(self.inv, selected, pinned.pids(),
                                           self.cfg.drm_major, self.cfg.busy_detection,
                                           kfd_root=self.cfg.kfd_proc_path if real else "",
                                           tables=not real or procs.host_pid_ns())
                    busy = {k: [p for p in v if not pinned.exited(p)] for k, v in busy.items()}
                    busy = {k: v for k, v in busy.items() if v}
            except (MountError, InjectedFault) as e:
                if pinned is not None:
                    pinned.close()
                if await self._rollback(pod, "detach"):   # the pod went away meanwhile
                    return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_POD_NOT_FOUND,
                                                 message=f"pod went away: {e}")
                raise RpcError(grpc.StatusCode.INTERNAL, f"{ERR_INTERNAL}: {e}") from e
            if busy and not req.force:
                pinned.close()
                _log.info("GPU busy in %s/%s: %s", req.namespace, req.pod_name, busy)
                return api.RemoveGPUResponse(
                    remove_gpu_result=api.REMOVE_BUSY,
                    message=f"busy: {json.dumps({str(k): v for k, v in busy.items()})}")
            phs = [ph for ph in st.placeholders
                   if {g.index for g in st.by_placeholder[(ph.namespace, ph.name)]} & sel_idx]
            killed: List[int] = sorted({p for v in busy.values() for p in v})
            survivors: List[int] = []
            held: List[Placeholder] = []
            try:
                # revoke, then kill, then release (reference order deny → rm → kill,
                # util.go:112-139, then slave deletion, server.go:170-175). The revoke only
                # gates open(): a killed process keeps its render/KFD fds until it has exited,
                # so the placeholder keeps the GPU booked until then (worker/drain.py)
                with trace.span("unmount", gpus=len(selected)):
                    self.hm.detach(pod, selected, keep, st.own, req.container, targets)
                if killed:
                    with trace.span("kill", pids=len(killed)):
                        try:    # GM_FAULT=kill_escalation:1: as if SIGKILL could not land yet
                            self.faults.check("kill_escalation")
                            sigkill = True
                        except InjectedFault:
                            sigkill = False
                        pinned.signal(killed, self.cfg.kill_signal)
                        _, survivors = await pinned.reap(
                            killed, self.cfg.kill_signal, self.cfg.kill_grace_s,
                            self.cfg.kill_reap_s, already_signalled=True, sigkill=sigkill)
                if survivors:
                    left = set(survivors)
                    stuck = {i for i, v in busy.items() if left.intersection(v)}
                    held = [ph for ph in phs if stuck & {
                        g.index for g in st.by_placeholder[(ph.namespace, ph.name)]}]
                    phs = [ph for ph in phs if ph not in held]
                    p, pinned = pinned, None
                    with trace.span("drain_hold", placeholders=len(held)):
                        # revoked and booked either way; a failed draining mark is retried
                        await self.drain.hold(pod, held, p, survivors)
                else:
                    pinned.close()
                    pinned = None
                await self._release(phs)
            except (MountError, ReserveError, InjectedFault, OSError) as e:
                if pinned is not None:
                    pinned.close()
                _log.error("detach failed on %s/%s: %s", req.namespace, req.pod_name, e)
                if await self._rollback(pod, "detach"):
                    return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_POD_NOT_FOUND,
                                                 message=f"pod went away: {e}")
                raise RpcError(grpc.StatusCode.INTERNAL, f"{ERR_INTERNAL}: {e}") from e
            owner = {g.index: ph.name for ph in phs + held
                     for g in st.by_placeholder[(ph.namespace, ph.name)]}
            log.kv(_log, 20, "detached", pod=f"{req.namespace}/{req.pod_name}",
                   gpus=[g.bdf for g in selected], killed=killed, by=req.requested_by,
                   still_running=survivors)
            self.notify.detached(pod, selected, keep, killed, by=req.requested_by)
            if survivors:
                gone = {g.index for ph in held for g in st.by_placeholder[(ph.namespace, ph.name)]}
                uuids = [g.uuid for g in selected if g.index in gone]
                return api.RemoveGPUResponse(
                    remove_gpu_result=api.REMOVE_BUSY, devices=self._devices(selected, owner),
                    killed_pids=killed,
                    message=f"busy: processes {survivors} still running "
                            f"{self.cfg.kill_reap_s:g}s after SIGKILL; access to {uuids} is "
                            f"revoked and they stay reserved until those processes exit")
            return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_SUCCESS,
                                         devices=self._devices(selected, owner),
                                         killed_pids=killed, message="Remove GPU Success")

    select_removal = staticmethod(planning.select_removal)

    # ------------------------------------------------------------------------ status
    async def node_status(self, include_processes: bool) -> dict:
        return await status.node_status(self, include_processes)
