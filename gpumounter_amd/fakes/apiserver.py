"""Hermetic kube-apiserver + scheduler + kubelet emulation for tests and benchmarks.

Serves the subset of the core/v1 Pod API the controller uses (GET/LIST/WATCH/POST/DELETE/PATCH,
label + field selectors, resourceVersion-based watch resume), and runs a tiny control loop:

* **scheduler** — binds pods to nodes whose labels match ``nodeSelector`` and whose extended
  resource capacity (``amd.com/gpu``) still fits; otherwise sets ``PodScheduled=False,
  reason=Unschedulable`` (what the reference waits for: allocator.go:266) and re-queues the pod
  when capacity frees up;
* **kubelet** — admits bound pods (device-plugin Allocate → PodResources ledger), pulls images
  (``Always`` pulls every time, ``IfNotPresent`` once per node), starts containers (cgroup +
  rootfs artifacts on the :class:`FakeNode`), honours grace periods and finalizers on delete;
* **garbage collector** — ownerReference cascade; in ``modern`` mode (Kubernetes ≥1.20) a
  dependent whose owner lives in another namespace is treated as ownerless and collected, which is
  exactly the hazard of the reference's cross-namespace slave pods (SURVEY §2.6 defect 4).

Every phase has an optional latency (:class:`LatencyModel`) so benchmarks can model a real
control plane; the default is zero (pure plumbing).
"""
from __future__ import annotations

import asyncio
import base64
import json
import secrets
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from aiohttp import web

from gpumounter_amd.fakes.node import FakeNode
from gpumounter_amd.models import pod as podu
from gpumounter_amd.utils import log

_log = log.get("fake.apiserver")


@dataclass
class LatencyModel:
    """Control-plane delays in milliseconds (0 = instantaneous)."""

    api_ms: float = 0.0        # every API request
    schedule_ms: float = 0.0   # create → bind
    admit_ms: float = 0.0      # bind → device-plugin Allocate (ledger visible)
    sandbox_ms: float = 0.0    # pod sandbox (pause container, CNI)
    pull_ms: float = 0.0       # image pull when required by pull policy
    start_ms: float = 0.0      # container start → Running
    stop_ms: float = 0.0       # SIGTERM → exit for images that handle SIGTERM
    # a deleted Pod → its containers and sandbox stopped on the node: until then the kubelet
    # counts it active and its devices stay allocated (0 = the next loop turn)
    teardown_ms: float = 0.0
    grace_scale: float = 0.0   # fraction of terminationGracePeriodSeconds waited when an image
                               # ignores SIGTERM (1.0 = real time)

    @classmethod
    def realistic(cls) -> "LatencyModel":
        """Order-of-magnitude figures for a small on-prem cluster (documented in BASELINE.md)."""
        return cls(api_ms=1.0, schedule_ms=10.0, admit_ms=15.0, sandbox_ms=300.0, pull_ms=1200.0,
                   start_ms=120.0, stop_ms=50.0, grace_scale=1.0, teardown_ms=50.0)


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


DEVICECLASS_QUOTA_SUFFIX = ".deviceclass.resource.k8s.io/devices"


def _parse_selector(sel: str):
    """Label selector → list of (key, op, value) with op in {=, !=, exists, !exists}."""
    out = []
    for part in filter(None, (p.strip() for p in (sel or "").split(","))):
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in part:
            k, v = part.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in part:
            k, v = part.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        elif part.startswith("!"):
            out.append((part[1:], "!exists", ""))
        else:
            out.append((part, "exists", ""))
    return out


def _match_labels(labels: Dict[str, str], sel) -> bool:
    for k, op, v in sel:
        if op == "=" and labels.get(k) != v:
            return False
        if op == "!=" and labels.get(k) == v:
            return False
        if op == "exists" and k not in labels:
            return False
        if op == "!exists" and k in labels:
            return False
    return True


def _field(pod: dict, key: str) -> str:
    cur: Any = pod
    for part in key.split("."):
        cur = cur.get(part, "") if isinstance(cur, dict) else ""
    return cur or ""


def _match_fields(pod: dict, sel) -> bool:
    for k, op, v in sel:
        if op == "=" and _field(pod, k) != v:
            return False
        if op == "!=" and _field(pod, k) == v:
            return False
    return True


def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return podu.jcopy(patch)
    if not isinstance(target, dict):
        target = {}
    for k, v in patch.items():
        if v is None:
            target.pop(k, None)
        else:
            target[k] = merge_patch(target.get(k), v)
    return target


class FakeCluster:
    """State + control loops; :meth:`app` exposes it over HTTP."""

    HISTORY = 20000
    EVENTS_KEPT = 5000        # core/v1 Events retained

    def __init__(self, latency: Optional[LatencyModel] = None, gc_mode: str = "modern") -> None:
        self.latency = latency or LatencyModel()
        self.gc_mode = gc_mode
        self.nodes: Dict[str, FakeNode] = {}
        self.pods: Dict[Tuple[str, str], dict] = {}
        self.rv = 1000
        self.events: List[Tuple[int, str, dict]] = []
        self.k8s_events: List[dict] = []     # core/v1 Event objects (not the watch history)
        self.quotas: Dict[Tuple[str, str], dict] = {}   # ResourceQuota objects (spec.hard)
        # ResourceQuota watch: the quota controller's status.used updates, as events
        self.quota_events: List[Tuple[int, str, bytes]] = []
        self.quota_watchers: List[Tuple[asyncio.Queue, str, Any, Any]] = []
        self.tokens: Dict[str, dict] = {}    # TokenReview: bearer token → user info
        self.rbac: List[dict] = []           # SubjectAccessReview rules (see grant())
        self.sar_count = 0
        self.ssar_count = 0
        self.serve_self_review = True     # False: /selfsubjectaccessreviews answers 404
        self.watchers: List[Tuple[asyncio.Queue, str, Any, Any]] = []
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.request_count = 0
        self.requests_by_verb: Dict[str, int] = {}
        self._unschedulable: set = set()
        self._handed_to_kubelet: set = set()   # pod UIDs bound and passed to kubelet admission
        self._tasks: set = set()
        self._lock = threading.RLock()
        self._faults: List[Tuple[str, int, bool, str]] = []
        self._random_faults: Optional[Tuple[float, Any]] = None   # (rate, random.Random)
        self.random_faults_served = 0
        self.last_fault_at = 0.0    # time.monotonic() when an injected failure was last served
        # every pod watch event reaches its watchers this much later (a slow watch cache, a
        # congested apiserver); order is kept
        self.watch_delay_s = 0.0
        from gpumounter_amd.fakes.dra import DraState
        self.dra = DraState(self)     # resource.k8s.io/v1 claims and slices (fakes/dra.py)
        # scheduling.k8s.io/v1 PriorityClasses: the two every cluster has; the harness applies
        # the shipped deploy's classes on top (deploy/placeholder-priority.yaml)
        self.priority_classes: Dict[str, dict] = {}
        self.add_priority_class("system-cluster-critical", 2000000000)
        self.add_priority_class("system-node-critical", 2000001000)
        self.preemptions = 0          # victims the scheduler evicted for a higher-priority Pod
        self.victims: List[dict] = []  # each victim as it was when preempted (last 1000)
        # Pod LISTs: pages served, the largest response body, and a switch that makes the next
        # continue tokens expire (410), as after an etcd compaction
        self.list_pages = 0
        self.max_list_bytes = 0
        self.expire_continue = False

    # ------------------------------------------------------------------------ nodes
    def add_node(self, node: FakeNode) -> FakeNode:
        self.nodes[node.name] = node
        return node

    # ------------------------------------------------------------------------ priority
    def add_priority_class(self, name: str, value: int,
                           preemption_policy: str = "PreemptLowerPriority",
                           global_default: bool = False, description: str = "") -> dict:
        pc = {"apiVersion": "scheduling.k8s.io/v1", "kind": "PriorityClass",
              "metadata": {"name": name, "uid": str(uuid.uuid4())}, "value": int(value),
              "preemptionPolicy": preemption_policy, "globalDefault": bool(global_default)}
        if description:
            pc["description"] = description
        self.priority_classes[name] = pc
        return pc

    def apply_priority_classes(self, docs) -> List[str]:
        """Create the PriorityClass objects among ``docs`` (parsed manifests), as
        ``kubectl apply`` of the deploy would; returns their names."""
        out = []
        for d in docs:
            if isinstance(d, dict) and d.get("kind") == "PriorityClass":
                self.add_priority_class(d["metadata"]["name"], int(d["value"]),
                                        d.get("preemptionPolicy") or "PreemptLowerPriority",
                                        bool(d.get("globalDefault")), d.get("description", ""))
                out.append(d["metadata"]["name"])
        return out

    def _priority_admit(self, pod: dict) -> None:
        """The Priority admission plugin: ``spec.priority`` and ``spec.preemptionPolicy`` come
        from the PriorityClass named (or the global default); a Pod naming a class that does
        not exist, or giving values that differ from the class's, is refused with 403."""
        spec = pod.setdefault("spec", {})
        pname = pod.get("metadata", {}).get("name", "")
        name = spec.get("priorityClassName") or ""
        if not name:
            d = next((c for c in self.priority_classes.values() if c.get("globalDefault")), None)
            if d is not None:
                name = spec["priorityClassName"] = d["metadata"]["name"]
        value, policy = 0, "PreemptLowerPriority"
        if name:
            pc = self.priority_classes.get(name)
            if pc is None:
                raise self._forbidden(f'pods "{pname}" is forbidden: no PriorityClass with '
                                      f"name {name} was found")
            value, policy = int(pc["value"]), pc.get("preemptionPolicy") or policy
        if spec.get("priority") is not None and int(spec["priority"]) != value:
            raise self._forbidden(
                f'pods "{pname}" is forbidden: the integer value of priority '
                f'({spec["priority"]}) must not be provided in pod spec; priority admission '
                f"controller computed {value} from the given PriorityClass name")
        if spec.get("preemptionPolicy") and spec["preemptionPolicy"] != policy:
            raise self._forbidden(
                f'pods "{pname}" is forbidden: the string value of PreemptionPolicy '
                f'({spec["preemptionPolicy"]}) must not be provided in pod spec; priority '
                f"admission controller computed {policy} from the given PriorityClass name")
        spec["priority"] = value
        spec["preemptionPolicy"] = policy

    @staticmethod
    def _forbidden(msg: str) -> web.HTTPForbidden:
        return web.HTTPForbidden(text=json.dumps({"kind": "Status", "reason": "Forbidden",
                                                  "code": 403, "message": msg}),
                                 content_type="application/json")

    # ------------------------------------------------------------------------ events
    def _bump(self, etype: str, pod: dict) -> None:
        self.rv += 1
        pod["metadata"]["resourceVersion"] = str(self.rv)
        # history and watch queues hold the serialized object: bytes are not tracked by the
        # cyclic GC, so a long history does not turn into long collector pauses in this
        # stand-in for the (Go) apiserver
        data = json.dumps(pod).encode()
        self.events.append((self.rv, etype, data))
        if len(self.events) > self.HISTORY:
            del self.events[: len(self.events) - self.HISTORY]
        t = time.monotonic()
        for q, ns, lsel, fsel in list(self.watchers):
            if self._matches(pod, ns, lsel, fsel):
                q.put_nowait((etype, data, t))
        if self.quotas:
            self.quota_touch(pod["metadata"].get("namespace", ""))

    @staticmethod
    def _matches(pod: dict, ns: str, lsel, fsel) -> bool:
        if ns and pod["metadata"].get("namespace") != ns:
            return False
        return _match_labels(pod["metadata"].get("labels", {}) or {}, lsel) and \
            _match_fields(pod, fsel)

    def _spawn(self, coro) -> None:
        t = asyncio.ensure_future(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    # ------------------------------------------------------------------------ pod CRUD
    def create_pod(self, ns: str, body: dict, *, schedule: bool = True) -> dict:
        pod = podu.jcopy(body)
        md = pod.setdefault("metadata", {})
        if not md.get("name"):
            gen = md.get("generateName")
            if not gen:
                raise web.HTTPUnprocessableEntity(text=json.dumps(
                    {"kind": "Status", "message": "name or generateName is required"}))
            md["name"] = gen + secrets.token_hex(3)[:5]
        md["namespace"] = ns
        if (ns, md["name"]) in self.pods:
            raise web.HTTPConflict(text=json.dumps(
                {"kind": "Status", "reason": "AlreadyExists",
                 "message": f'pods "{md["name"]}" already exists'}), content_type="application/json")
        md["uid"] = str(uuid.uuid4())
        md["creationTimestamp"] = _now()
        md.setdefault("labels", {})
        md.setdefault("annotations", {})
        pod.setdefault("spec", {})
        self._priority_admit(pod)
        self._quota_admit(ns, pod)
        pod["status"] = {"phase": "Pending", "conditions": []}
        self.pods[(ns, md["name"])] = pod
        self._bump("ADDED", pod)
        if schedule:
            self._spawn(self._schedule(ns, md["name"]))
        return pod

    def get(self, ns: str, name: str) -> Optional[dict]:
        return self.pods.get((ns, name))

    # ------------------------------------------------------------------------ ResourceQuota
    def set_quota(self, ns: str, name: str, hard: Dict[str, str]) -> dict:
        q = {"apiVersion": "v1", "kind": "ResourceQuota",
             "metadata": {"name": name, "namespace": ns, "uid": str(uuid.uuid4())},
             "spec": {"hard": dict(hard)}}
        self.quotas[(ns, name)] = q
        self._quota_bump("ADDED", q)
        return q

    def _quota_bump(self, etype: str, q: dict) -> None:
        """A quota object changed, or its status.used did (the quota controller rewrites the
        status as the namespace's pods and claims change): an event for its watchers."""
        self.rv += 1
        q["metadata"]["resourceVersion"] = str(self.rv)
        data = json.dumps(self._quota_view(q)).encode()
        self.quota_events.append((self.rv, etype, data))
        if len(self.quota_events) > self.HISTORY:
            del self.quota_events[: len(self.quota_events) - self.HISTORY]
        t = time.monotonic()
        for wq, ns, lsel, fsel in list(self.quota_watchers):
            if self._matches(q, ns, lsel, fsel):
                wq.put_nowait((etype, data, t))

    def quota_touch(self, ns: str) -> None:
        """The namespace's usage may have changed: re-publish its quotas (no-op without)."""
        if not self.quotas:
            return
        for (qns, _), q in list(self.quotas.items()):
            if qns == ns:
                self._quota_bump("MODIFIED", q)

    def _quota_used(self, ns: str, key: str) -> int:
        """What the quota controller reports: requests of the namespace's non-terminal pods
        (extended resources: requests == limits)."""
        if key.endswith(DEVICECLASS_QUOTA_SUFFIX):    # DRA: devices of the namespace's claims
            return self.dra.quota_used(ns, key[:-len(DEVICECLASS_QUOTA_SUFFIX)])
        res = key[len("requests."):] if key.startswith("requests.") else key
        if "/" not in res:
            return 0
        return sum(podu.resource_limit(p, res) for (pns, _), p in self.pods.items()
                   if pns == ns and p.get("status", {}).get("phase") not in ("Succeeded", "Failed"))

    def _quota_view(self, q: dict) -> dict:
        out = podu.jcopy(q)
        ns = q["metadata"]["namespace"]
        out["status"] = {"hard": dict(q["spec"]["hard"]),
                         "used": {k: str(self._quota_used(ns, k)) for k in q["spec"]["hard"]}}
        return out

    def _quota_admit(self, ns: str, pod: dict) -> None:
        """The apiserver's ResourceQuota admission for extended resources."""
        for (qns, qname), q in self.quotas.items():
            if qns != ns:
                continue
            for key, hard in q["spec"]["hard"].items():
                res = key[len("requests."):] if key.startswith("requests.") else key
                want = podu.resource_limit(pod, res) if "/" in res else 0
                if want and self._quota_used(ns, key) + want > int(hard):
                    raise web.HTTPForbidden(text=json.dumps(
                        {"kind": "Status", "reason": "Forbidden", "code": 403,
                         "message": f'pods "{pod["metadata"].get("name")}" is forbidden: '
                                    f"exceeded quota: {qname}, requested: {key}={want}, used: "
                                    f"{key}={self._quota_used(ns, key)}, limited: {key}={hard}"}),
                        content_type="application/json")

    def _used(self, node: str, resource: str, exclude: Tuple[str, str] = ("", "")) -> int:
        total = 0
        for key, p in self.pods.items():
            if key == exclude or podu.node_of(p) != node:
                continue
            if p["status"].get("phase") in ("Succeeded", "Failed"):
                continue
            total += podu.resource_limit(p, resource)
        return total

    def _nominated(self, node: str, resource: str, pod: dict) -> int:
        """What Pods nominated to ``node`` by a preemption (not bound yet) need, counted
        against ``pod`` when they rank at least as high: the scheduler keeps the room a
        preemption freed for the preemptor, so a lower-priority Pod cannot take it back."""
        prio, me = podu.priority_of(pod), podu.uid_of(pod)
        return sum(podu.resource_limit(p, resource) for p in self.pods.values()
                   if podu.nominated_node(p) == node and not podu.node_of(p)
                   and podu.uid_of(p) != me and podu.priority_of(p) >= prio
                   and not podu.is_terminating(p))

    def _victims(self, pod: dict, node: FakeNode) -> Optional[List[dict]]:
        """The fewest lowest-priority Pods on ``node`` whose eviction makes ``pod`` fit (Pods of
        lower priority only; those already terminating count as gone): None if even evicting
        all of them would not."""
        prio = podu.priority_of(pod)
        want = podu.resource_limit(pod, node.resource)
        need = self._used(node.name, node.resource, (podu.ns_of(pod), podu.name_of(pod))) + \
            self._nominated(node.name, node.resource, pod) + want - node.capacity
        cands = sorted((p for p in self.pods.values()
                        if podu.node_of(p) == node.name and not podu.is_terminating(p)
                        and p["status"].get("phase") not in ("Succeeded", "Failed")
                        and podu.priority_of(p) < prio
                        and podu.resource_limit(p, node.resource) > 0),
                       key=lambda p: (podu.priority_of(p),
                                      p["metadata"].get("creationTimestamp", "")))
        out: List[dict] = []
        for p in cands:
            if need <= 0:
                break
            out.append(p)
            need -= podu.resource_limit(p, node.resource)
        return out if need <= 0 else None

    def _preempt(self, pod: dict, nodes: List[FakeNode]) -> str:
        """Default preemption: on the node where it costs least (lowest highest-victim
        priority, then fewest victims), evict lower-priority Pods with a DisruptionTarget
        condition and their own grace period, and nominate the node for ``pod``; it is bound
        when the victims are gone (the retry on freed capacity). Returns the message suffix."""
        if podu.nominated_node(pod):
            return f"; waiting for preemption on {podu.nominated_node(pod)}"
        best = None
        for n in nodes:
            v = self._victims(pod, n)
            if v:
                cost = (max(podu.priority_of(p) for p in v), len(v))
                if best is None or cost < best[0]:
                    best = (cost, n, v)
        if best is None:
            return "; preemption: no lower-priority victims would make room"
        _, node, victims = best
        pod["status"]["nominatedNodeName"] = node.name
        for v in victims:
            conds = v["status"].setdefault("conditions", [])
            conds.append({"type": "DisruptionTarget", "status": "True",
                          "reason": "PreemptionByScheduler",
                          "message": f"{podu.ns_of(pod)}: preempting to accommodate a higher "
                                     f"priority pod", "lastTransitionTime": _now()})
            self._bump("MODIFIED", v)
            self.preemptions += 1
            self.victims = self.victims[-999:] + [podu.jcopy(v)]
            _log.info("preempting %s/%s (priority %d) for %s/%s (priority %d)",
                      podu.ns_of(v), podu.name_of(v), podu.priority_of(v), podu.ns_of(pod),
                      podu.name_of(pod), podu.priority_of(pod))
            self.delete(podu.ns_of(v), podu.name_of(v))
        return f"; preempting {len(victims)} pod(s) on {node.name}"

    async def _sleep(self, ms: float) -> None:
        if ms > 0:
            await asyncio.sleep(ms / 1e3)

    async def _schedule(self, ns: str, name: str) -> None:
        pod = self.pods.get((ns, name))
        direct = pod is not None and bool(podu.node_of(pod)) and not self.dra.refs(pod)
        if not direct:
            # a Pod created with spec.nodeName is the kubelet's at once: no scheduling cycle
            await self._sleep(self.latency.schedule_ms)
        pod = self.pods.get((ns, name))
        if pod is None or podu.is_terminating(pod):
            return
        uid = pod["metadata"]["uid"]
        if uid in self._handed_to_kubelet:
            # several capacity-freed retries can be queued for one unschedulable pod; a pod is
            # bound and admitted once (a second admission would Allocate devices again)
            return
        if self.dra.refs(pod):
            # DRA: the scheduler allocates the Pod's claims on a node, then binds it there
            sel = pod["spec"].get("nodeSelector", {}) or {}
            cands = [n for n in self.nodes.values()
                     if all(n.labels.get(k) == v for k, v in sel.items())
                     and (not podu.node_of(pod) or n.name == podu.node_of(pod))]
            node_name, why = self.dra.schedule(pod, cands)
            if not node_name:
                pod["status"]["conditions"] = [{
                    "type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                    "message": f"0/{len(self.nodes)} nodes are available: {why}",
                    "lastTransitionTime": _now()}]
                self._unschedulable.add((ns, name))
                self._bump("MODIFIED", pod)
                return
            pod["spec"]["nodeName"] = node_name
        elif podu.node_of(pod):
            node_name = podu.node_of(pod)
            n = self.nodes.get(node_name)
            if n is not None and direct:
                # the kubelet's own admission (GeneralPredicates): what the Pods bound to the
                # node request, against its capacity; nominations are the scheduler's business
                want = podu.resource_limit(pod, n.resource)
                used = self._used(n.name, n.resource, (ns, name))
                if want and used + want > n.capacity:
                    pod["status"]["phase"] = "Failed"
                    pod["status"]["reason"] = f"OutOf{n.resource}"
                    pod["status"]["message"] = (
                        f"Pod was rejected: Node didn't have enough resource: {n.resource}, "
                        f"requested: {want}, used: {used}, capacity: {n.capacity}")
                    self._bump("MODIFIED", pod)
                    return
        else:
            sel = pod["spec"].get("nodeSelector", {}) or {}
            node_name = ""
            fits = [n for n in self.nodes.values()
                    if all(n.labels.get(k) == v for k, v in sel.items())]
            for n in fits:
                want = podu.resource_limit(pod, n.resource)
                if self._used(n.name, n.resource, (ns, name)) + \
                        self._nominated(n.name, n.resource, pod) + want <= n.capacity:
                    node_name = n.name
                    break
            if not node_name:
                why = "insufficient resources"
                if pod["spec"].get("preemptionPolicy", "PreemptLowerPriority") != "Never":
                    why += self._preempt(pod, fits)
                elif any(self._victims(pod, n) is not None for n in fits):
                    why += "; preemption is not allowed for this Pod (preemptionPolicy Never)"
                pod["status"]["conditions"] = [{
                    "type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                    "message": "0/%d nodes are available: %s" % (len(self.nodes), why),
                    "lastTransitionTime": _now()}]
                self._unschedulable.add((ns, name))
                self._bump("MODIFIED", pod)
                return
            pod["spec"]["nodeName"] = node_name
            pod["status"].pop("nominatedNodeName", None)
        self._unschedulable.discard((ns, name))
        pod["status"]["conditions"] = [{"type": "PodScheduled", "status": "True",
                                        "lastTransitionTime": _now()}]
        self._bump("MODIFIED", pod)
        self._handed_to_kubelet.add(uid)
        self._spawn(self._kubelet_run(ns, name, node_name))

    async def _kubelet_run(self, ns: str, name: str, node_name: str) -> None:
        node = self.nodes.get(node_name)
        if node is None:
            return
        await self._sleep(self.latency.admit_ms)
        pod = self.pods.get((ns, name))
        if pod is None or podu.is_terminating(pod):
            return
        # device-plugin Allocate per container (admission)
        for c in pod["spec"].get("containers", []):
            want = int(podu.parse_quantity(
                ((c.get("resources") or {}).get("limits") or {}).get(node.resource, 0)))
            if want:
                # the kubelet hands a device plugin the pod's UID and container name, never its
                # annotations: gpumounter's preferred-devices hint does not reach it
                if node.plugin is not None:      # kubelet device manager → device plugin
                    ids = await node.plugin.plugin_allocate(ns, name, c["name"], want,
                                                            uid=pod["metadata"]["uid"])
                else:
                    ids = node.allocate(ns, name, c["name"], want, uid=pod["metadata"]["uid"])
                if ids is None:
                    node.release_pod(ns, name)
                    pod["status"]["phase"] = "Failed"
                    pod["status"]["reason"] = "UnexpectedAdmissionError"
                    self._bump("MODIFIED", pod)
                    return
                if self.pods.get((ns, name)) is not pod:   # deleted while the plugin ran
                    node.release_pod(ns, name)
                    return
        pod["status"]["containerStatuses"] = [
            {"name": c["name"], "ready": False, "restartCount": 0, "image": c.get("image", ""),
             "state": {"waiting": {"reason": "ContainerCreating"}}}
            for c in pod["spec"].get("containers", [])]
        self._bump("MODIFIED", pod)
        await self._sleep(self.latency.sandbox_ms)
        for c in pod["spec"].get("containers", []):
            img = c.get("image", "")
            policy = c.get("imagePullPolicy") or ("Always" if img.endswith(":latest") or
                                                  ":" not in img else "IfNotPresent")
            if policy == "Always" or (policy == "IfNotPresent" and img not in node.images):
                await self._sleep(self.latency.pull_ms)
                node.images.add(img)
        await self._sleep(self.latency.start_ms)
        pod = self.pods.get((ns, name))
        if pod is None or podu.is_terminating(pod):
            return
        self._start_containers(node, pod)

    def _start_containers(self, node: FakeNode, pod: dict, pids=None) -> None:
        statuses = []
        for c in pod["spec"].get("containers", []):
            ctr = node.start_container(pod, c["name"], (pids or {}).get(c["name"], ()))
            statuses.append({
                "name": c["name"], "ready": True, "restartCount": 0, "image": c.get("image", ""),
                "containerID": f"{node.runtime}://{ctr.id}",
                "state": {"running": {"startedAt": _now()}}})
        pod["status"]["containerStatuses"] = statuses
        pod["status"]["phase"] = "Running"
        pod["status"]["podIP"] = pod["status"].get("podIP") or "10.0.0.%d" % (self.rv % 250 + 2)
        pod["status"]["conditions"] = [
            {"type": "PodScheduled", "status": "True"}, {"type": "Ready", "status": "True"}]
        pod["status"]["qosClass"] = podu.qos_class(pod)
        self._bump("MODIFIED", pod)

    def restart_container(self, ns: str, name: str, cname: str) -> str:
        """The container exits and the kubelet starts it again (restartPolicy Always): a new
        container id, cgroup and root filesystem — no device gpumounter added survives — and a
        MODIFIED event with restartCount + 1. Returns the new container id."""
        with self._lock:
            pod = self.pods[(ns, name)]
            node = self.nodes[pod["spec"]["nodeName"]]
            cs = next(c for c in pod["status"]["containerStatuses"] if c["name"] == cname)
            old = cs["containerID"].split("://", 1)[1]
            octr = node.container(old)
            pids = octr.pids if octr is not None else []
            node.stop_container(old)
            ctr = node.start_container(pod, cname, pids)
            cs.update({"containerID": f"{node.runtime}://{ctr.id}",
                       "restartCount": int(cs.get("restartCount", 0)) + 1,
                       "lastState": {"terminated": {"exitCode": 1, "finishedAt": _now()}},
                       "state": {"running": {"startedAt": _now()}}})
            self._bump("MODIFIED", pod)
            return ctr.id

    def create_running_pod(self, ns: str, body: dict, node: str,
                           pids: Optional[Dict[str, List[int]]] = None,
                           pod_ip: str = "") -> dict:
        """Test helper: a tenant pod that is already bound, admitted and running (at
        ``pod_ip`` from its first Running version on, when given)."""
        pod = self.create_pod(ns, body, schedule=False)
        pod["spec"]["nodeName"] = node
        if pod_ip:
            pod["status"]["podIP"] = pod_ip
        n = self.nodes[node]
        for c in pod["spec"].get("containers", []):
            want = int(podu.parse_quantity(
                ((c.get("resources") or {}).get("limits") or {}).get(n.resource, 0)))
            if want and n.allocate(ns, pod["metadata"]["name"], c["name"], want,
                                   uid=pod["metadata"]["uid"]) is None:
                raise RuntimeError("tenant pod does not fit")
        self._start_containers(n, pod, pids)
        return pod

    def delete(self, ns: str, name: str, grace: Optional[int] = None,
               uid_precondition: str = "", rv_precondition: str = "") -> Optional[dict]:
        pod = self.pods.get((ns, name))
        if pod is None:
            return None
        if uid_precondition and pod["metadata"]["uid"] != uid_precondition:
            raise web.HTTPConflict(text=json.dumps({"kind": "Status", "message": "uid mismatch"}),
                                   content_type="application/json")
        if rv_precondition and pod["metadata"].get("resourceVersion") != rv_precondition:
            raise web.HTTPConflict(text=json.dumps({
                "kind": "Status", "message": "resourceVersion mismatch"}),
                content_type="application/json")
        if grace is None:
            grace = int(pod["spec"].get("terminationGracePeriodSeconds", 30))
        md = pod["metadata"]
        if not md.get("deletionTimestamp"):
            md["deletionTimestamp"] = _now()
            md["deletionGracePeriodSeconds"] = grace
            self._bump("MODIFIED", pod)
        running = pod["status"].get("phase") == "Running"
        if grace == 0 or not running:
            self._maybe_finalize(ns, name)
        else:
            self._spawn(self._terminate(ns, name, grace))
        return pod

    async def _terminate(self, ns: str, name: str, grace: int) -> None:
        pod = self.pods.get((ns, name))
        if pod is None:
            return
        if self._ignores_sigterm(pod):
            await asyncio.sleep(grace * self.latency.grace_scale)
        else:
            await self._sleep(self.latency.stop_ms)
        self._maybe_finalize(ns, name)

    @staticmethod
    def _ignores_sigterm(pod: dict) -> bool:
        # a `sh -c "while true; ...; sleep 10; done"` container (reference allocator.go:217-220)
        # runs as PID 1 without a SIGTERM handler, so the kubelet waits the whole grace period.
        for c in pod["spec"].get("containers", []):
            cmd = " ".join((c.get("command") or []) + (c.get("args") or []))
            if "while true" in cmd:
                return True
        return False

    def _maybe_finalize(self, ns: str, name: str) -> None:
        pod = self.pods.get((ns, name))
        if pod is None:
            return
        pod["status"]["phase"] = pod["status"].get("phase", "Pending")
        if pod["metadata"].get("finalizers"):
            return  # wait for the controller to drop finalizers (PATCH)
        self._remove(ns, name)

    def _remove(self, ns: str, name: str) -> None:
        pod = self.pods.pop((ns, name), None)
        if pod is None:
            return
        self._handed_to_kubelet.discard(pod["metadata"]["uid"])
        self.dra.pod_gone(pod)
        self._unschedulable.discard((ns, name))
        node = self.nodes.get(podu.node_of(pod))
        self._bump("DELETED", pod)
        self._gc(pod)
        # The apiserver answers the DELETE once the object is gone from storage; the kubelet
        # learns of it from its own watch and tears the pod down afterwards (containers,
        # device-manager entry, checkpoint). Modelled as the next loop turn: after this
        # request's reply, before any later request's admission (allocate() also frees it);
        # or, with latency.teardown_ms, that much later (the Pod stays active until then)
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:                 # no loop (synchronous test helpers)
            loop = None
        if loop is not None and self.latency.teardown_ms > 0:
            # by UID: the same name may be a new Pod by then (a re-created tenant)
            loop.call_later(self.latency.teardown_ms / 1e3, self._teardown, node, ns, name,
                            pod["metadata"]["uid"])
            return
        if node is not None:
            node.pending_release.add((ns, name))
        if loop is not None:
            loop.call_soon(self._teardown, node, ns, name)
        else:
            self._teardown(node, ns, name)

    def _teardown(self, node: Optional[FakeNode], ns: str, name: str, uid: str = "") -> None:
        if node is not None:
            node.release_pod(ns, name, uid)
            node.stop_pod_containers(ns, name, uid)
        # capacity freed: retry unschedulable pods (scheduler queue)
        for key in list(self._unschedulable):
            self._spawn(self._schedule(*key))

    def _gc(self, owner: dict) -> None:
        ouid = owner["metadata"]["uid"]
        for (ns, name), p in list(self.pods.items()):
            for ref in p["metadata"].get("ownerReferences", []) or []:
                if ref.get("uid") != ouid:
                    continue
                if self.gc_mode == "modern" and ns != owner["metadata"]["namespace"]:
                    continue  # handled by _gc_invalid_refs: owner was never visible
                self.delete(ns, name, grace=0)

    def gc_sweep(self) -> int:
        """Modern-GC rule: a namespaced owner must be in the dependent's namespace, otherwise the
        reference is treated as absent and the dependent is deleted. Returns #deleted."""
        n = 0
        for (ns, name), p in list(self.pods.items()):
            refs = p["metadata"].get("ownerReferences", []) or []
            if not refs:
                continue
            live = False
            for ref in refs:
                for (ons, oname), o in self.pods.items():
                    if o["metadata"]["uid"] == ref.get("uid") and \
                            (self.gc_mode == "legacy" or ons == ns):
                        live = True
            if not live:
                self.delete(ns, name, grace=0)
                n += 1
        return n

    def patch(self, ns: str, name: str, patch: dict) -> Optional[dict]:
        pod = self.pods.get((ns, name))
        if pod is None:
            return None
        md_patch = patch.get("metadata", {})
        want_rv = md_patch.get("resourceVersion")
        if want_rv is not None and want_rv != pod["metadata"].get("resourceVersion"):
            # a resourceVersion in the patch is a precondition (optimistic concurrency)
            raise web.HTTPConflict(text=json.dumps({
                "kind": "Status", "code": 409, "reason": "Conflict",
                "message": f'Operation cannot be fulfilled on pods "{name}": the object has '
                           "been modified; please apply your changes to the latest version "
                           "and try again"}), content_type="application/json")
        merged = merge_patch(pod["metadata"], md_patch)
        pod["metadata"] = merged
        if "spec" in patch:
            pod["spec"] = merge_patch(pod["spec"], patch["spec"])
        self._bump("MODIFIED", pod)
        if pod["metadata"].get("deletionTimestamp") and not pod["metadata"].get("finalizers"):
            running = pod["status"].get("phase") == "Running"
            if not running or pod["metadata"].get("deletionGracePeriodSeconds", 0) == 0:
                self._remove(ns, name)
        return pod

    # ------------------------------------------------------------------------ HTTP
    def app(self) -> web.Application:
        app = web.Application(client_max_size=8 << 20, middlewares=[self._fault_mw])
        r = app.router
        r.add_get("/api/v1/pods", self._h_list)
        r.add_get("/api/v1/namespaces/{ns}/pods", self._h_list)
        r.add_post("/api/v1/namespaces/{ns}/pods", self._h_create)
        r.add_get("/api/v1/namespaces/{ns}/pods/{name}", self._h_get)
        r.add_delete("/api/v1/namespaces/{ns}/pods/{name}", self._h_delete)
        r.add_patch("/api/v1/namespaces/{ns}/pods/{name}", self._h_patch)
        r.add_get("/api/v1/nodes", self._h_nodes)
        r.add_get("/api/v1/namespaces/{ns}/resourcequotas", self._h_quota_list)
        r.add_get("/api/v1/resourcequotas", self._h_quota_list)
        r.add_post("/apis/authentication.k8s.io/v1/tokenreviews", self._h_token_review)
        r.add_post("/apis/authorization.k8s.io/v1/subjectaccessreviews", self._h_sar)
        r.add_post("/apis/authorization.k8s.io/v1/selfsubjectaccessreviews", self._h_ssar)
        r.add_post("/api/v1/namespaces/{ns}/events", self._h_event_create)
        r.add_get("/api/v1/namespaces/{ns}/events", self._h_event_list)
        r.add_get("/healthz", self._h_healthz)
        r.add_get("/apis/scheduling.k8s.io/v1/priorityclasses", self._h_pc_list)
        r.add_get("/apis/scheduling.k8s.io/v1/priorityclasses/{name}", self._h_pc_get)
        r.add_post("/apis/scheduling.k8s.io/v1/priorityclasses", self._h_pc_create)
        self.dra.install(r, self._pre)
        return app

    async def _h_healthz(self, req: web.Request) -> web.Response:
        return web.Response(text="ok")

    def expire_watches(self) -> None:
        """Every open pod watch ends with 410 Gone (its resourceVersion left the history, as
        after an apiserver restart or a compaction): the clients relist."""
        t = time.monotonic()
        for q, _, _, _ in list(self.watchers):
            q.put_nowait(("__EXPIRE__", b"", t))

    def fail_next(self, method: str, status: int = 503, count: int = 1,
                  after: bool = False, path: str = "/pods") -> None:
        """Fault injection: the next ``count`` requests with ``method`` whose path contains
        ``path`` answer ``status``. ``after=True`` performs the request first and loses the
        response (a dropped reply)."""
        self._faults.extend([(method, status, after, path)] * count)

    def random_failures(self, rate: float, seed: int = 0) -> None:
        """Fault injection at random: each Pod or ResourceClaim request fails with probability
        ``rate``: 500, 503 or 429, half of them after the request took effect (a lost reply).
        Watch streams end early before an event with probability ``rate/4`` per event (one in
        five of those with 410 Gone, forcing a relist). ``rate=0`` turns it off."""
        import random
        self._random_faults = (rate, random.Random(seed)) if rate > 0 else None

    @web.middleware
    async def _fault_mw(self, request: web.Request, handler):
        """Serves the failures queued by :meth:`fail_next` (watch streams are never hit)."""
        rf = self._random_faults
        if rf is not None and not request.query.get("watch") and (
                "/pods" in request.path or "/resourceclaims" in request.path):
            rate, rnd = rf
            if rnd.random() < rate:
                self.random_faults_served += 1
                st = rnd.choice((500, 503, 429))
                if rnd.random() < 0.5:
                    await self._lost_reply(handler, request)
                return web.json_response({"kind": "Status", "code": st,
                                          "message": "injected failure"}, status=st)
        if self._faults and not request.query.get("watch"):
            for i, (m, st, after, path) in enumerate(self._faults):
                if m == request.method and path in request.path:
                    del self._faults[i]
                    self.last_fault_at = time.monotonic()
                    if after:
                        await self._lost_reply(handler, request)
                    return web.json_response({"kind": "Status", "code": st,
                                              "message": "injected failure"}, status=st)
        return await handler(request)

    @staticmethod
    async def _lost_reply(handler, request: web.Request) -> None:
        """The request is served (or refused: a conflict, a missing object), and whatever it
        answered gets lost on the way back."""
        try:
            await handler(request)
        except web.HTTPException:
            pass

    async def _pre(self, req: web.Request) -> None:
        self.request_count += 1
        kind = "watch" if req.query.get("watch") else ("events" if "/events" in req.path else "")
        key = f"{req.method} {kind}".strip()   # pod verbs stay "GET"/"POST"/...
        self.requests_by_verb[key] = self.requests_by_verb.get(key, 0) + 1
        await self._sleep(self.latency.api_ms)

    @staticmethod
    def _not_found(ns: str, name: str) -> web.Response:
        return web.json_response({"kind": "Status", "status": "Failure", "reason": "NotFound",
                                  "message": f'pods "{name}" not found', "code": 404}, status=404)

    async def _h_get(self, req: web.Request) -> web.Response:
        await self._pre(req)
        ns, name = req.match_info["ns"], req.match_info["name"]
        pod = self.pods.get((ns, name))
        if pod is None:
            return self._not_found(ns, name)
        return web.json_response(pod)

    async def _h_list(self, req: web.Request):
        await self._pre(req)
        ns = req.match_info.get("ns", "")
        lsel = _parse_selector(req.query.get("labelSelector", ""))
        fsel = _parse_selector(req.query.get("fieldSelector", ""))
        if req.query.get("watch") in ("true", "1"):
            return await self._watch(req, ns, lsel, fsel)
        limit = int(req.query.get("limit", "0") or 0)
        cont = req.query.get("continue", "")
        rv, after = str(self.rv), None
        if cont:
            try:
                tok = json.loads(base64.urlsafe_b64decode(cont.encode()))
                rv, after = tok["rv"], tuple(tok["key"])
            except (ValueError, KeyError, TypeError):
                return web.json_response({"kind": "Status", "code": 400, "reason": "BadRequest",
                                          "message": "invalid continue token"}, status=400)
            if self.events and int(rv) < self.events[0][0] - 1 or self.expire_continue:
                # the snapshot the token points into was compacted
                return web.json_response(
                    {"kind": "Status", "code": 410, "reason": "Expired",
                     "message": "The provided continue parameter is too old to display a "
                                "consistent list result."}, status=410)
        keys = sorted(k for k, p in self.pods.items() if self._matches(p, ns, lsel, fsel)
                      and (after is None or k > after))
        md = {"resourceVersion": rv}
        if limit and len(keys) > limit:
            keys = keys[:limit]
            md["continue"] = base64.urlsafe_b64encode(json.dumps(
                {"rv": rv, "key": list(keys[-1])}).encode()).decode()
        body = json.dumps({"kind": "PodList", "apiVersion": "v1", "metadata": md,
                           "items": [self.pods[k] for k in keys]}).encode()
        self.list_pages += 1
        self.max_list_bytes = max(self.max_list_bytes, len(body))
        return web.Response(body=body, content_type="application/json")

    async def _watch(self, req: web.Request, ns: str, lsel, fsel, history=None, watchers=None,
                     current=None, kind: str = "Pod") -> web.StreamResponse:
        """A watch stream over ``history`` (rv, type, object) and live events queued through
        ``watchers``; pods by default, any collection (DRA claims) when given."""
        history = self.events if history is None else history
        watchers = self.watchers if watchers is None else watchers
        current = (lambda: list(self.pods.values())) if current is None else current
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        await resp.prepare(req)
        q: asyncio.Queue = asyncio.Queue()
        rv = req.query.get("resourceVersion", "")
        if rv and rv != "0":
            since = int(rv)
            if history and since < history[0][0] - 1:
                await resp.write(json.dumps({"type": "ERROR", "object": {
                    "kind": "Status", "code": 410, "reason": "Expired",
                    "message": "too old resource version"}}).encode() + b"\n")
                return resp
            for erv, et, data in history:
                if erv > since and self._matches(json.loads(data), ns, lsel, fsel):
                    q.put_nowait((et, data))
        else:
            for p in current():
                if self._matches(p, ns, lsel, fsel):
                    q.put_nowait(("ADDED", json.dumps(p).encode()))
        entry = (q, ns, lsel, fsel)
        watchers.append(entry)
        timeout = float(req.query.get("timeoutSeconds", "300"))
        deadline = time.monotonic() + timeout
        idle = 0.0
        try:
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                if req.transport is None or req.transport.is_closing():
                    break  # client went away
                try:
                    item = await asyncio.wait_for(q.get(), timeout=min(left, 0.5))
                except asyncio.TimeoutError:
                    idle += 0.5
                    if idle >= 30:
                        idle = 0.0
                        await resp.write(json.dumps({"type": "BOOKMARK", "object": {
                            "kind": kind, "metadata": {"resourceVersion": str(self.rv)}}}
                        ).encode() + b"\n")
                    continue
                idle = 0.0
                et, obj = item[0], item[1]
                if et == "__EXPIRE__":
                    await resp.write(json.dumps({"type": "ERROR", "object": {
                        "kind": "Status", "code": 410, "reason": "Expired",
                        "message": "too old resource version"}}).encode() + b"\n")
                    break
                if len(item) > 2 and self.watch_delay_s > 0:
                    lag = item[2] + self.watch_delay_s - time.monotonic()
                    if lag > 0:
                        await asyncio.sleep(lag)
                rf = self._random_faults
                if rf is not None and rf[1].random() < rf[0] / 4:
                    # random_failures also disrupts watches: the stream ends before this event
                    # (the client resumes from its last resourceVersion) or, rarer, answers 410
                    # Gone (the client relists)
                    self.random_faults_served += 1
                    if rf[1].random() < 0.2:
                        await resp.write(json.dumps({"type": "ERROR", "object": {
                            "kind": "Status", "code": 410, "reason": "Expired",
                            "message": "injected: too old resource version"}}).encode() + b"\n")
                    break
                await resp.write(b'{"type": "' + et.encode() + b'", "object": ' + obj + b"}\n")
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            if entry in watchers:
                watchers.remove(entry)
        return resp

    async def _h_create(self, req: web.Request) -> web.Response:
        await self._pre(req)
        ns = req.match_info["ns"]
        body = await req.json()
        if req.query.get("dryRun") == "All":
            # validated and admitted (quota included), nothing stored, no watch event
            pod = podu.jcopy(body)
            md = pod.setdefault("metadata", {})
            md["namespace"] = ns
            md.setdefault("uid", str(uuid.uuid4()))
            self._priority_admit(pod)
            self._quota_admit(ns, pod)
            pod["status"] = {"phase": "Pending"}
            return web.json_response(pod, status=201)
        pod = self.create_pod(ns, body)
        return web.json_response(pod, status=201)

    async def _h_delete(self, req: web.Request) -> web.Response:
        await self._pre(req)
        ns, name = req.match_info["ns"], req.match_info["name"]
        grace = None
        uid = rv = ""
        if req.can_read_body:
            try:
                opts = await req.json()
            except ValueError:
                opts = {}
            if opts.get("gracePeriodSeconds") is not None:
                grace = int(opts["gracePeriodSeconds"])
            uid = (opts.get("preconditions") or {}).get("uid", "")
            rv = (opts.get("preconditions") or {}).get("resourceVersion", "")
        if "gracePeriodSeconds" in req.query:
            grace = int(req.query["gracePeriodSeconds"])
        pod = self.delete(ns, name, grace, uid, rv)
        if pod is None:
            return self._not_found(ns, name)
        return web.json_response(pod)

    async def _h_patch(self, req: web.Request) -> web.Response:
        await self._pre(req)
        ns, name = req.match_info["ns"], req.match_info["name"]
        pod = self.patch(ns, name, await req.json())
        if pod is None:
            return self._not_found(ns, name)
        return web.json_response(pod)

    # ------------------------------------------------------------------------ authn / authz
    def add_user(self, token: str, username: str, groups=()) -> None:
        self.tokens[token] = {"username": username, "uid": f"uid-{username}",
                              "groups": list(groups) + ["system:authenticated"]}

    def grant(self, subject: str, verbs, resource: str = "pods/gpumount",
              namespaces=("*",)) -> None:
        """RBAC-like rule: ``subject`` is a username or ``group:<name>``."""
        self.rbac.append({"subject": subject, "verbs": set(verbs), "resource": resource,
                          "namespaces": set(namespaces)})

    async def _h_token_review(self, req: web.Request) -> web.Response:
        await self._pre(req)
        body = await req.json()
        user = self.tokens.get(body.get("spec", {}).get("token", ""))
        status = {"authenticated": user is not None}
        if user is not None:
            status["user"] = user
        return web.json_response({**body, "status": status}, status=201)

    async def _h_sar(self, req: web.Request) -> web.Response:
        await self._pre(req)
        body = await req.json()
        spec = body.get("spec", {})
        allowed = self._allowed(spec.get("user", ""), spec.get("groups", []),
                                spec.get("resourceAttributes", {}))
        self.sar_count += 1
        return web.json_response({**body, "status": {"allowed": allowed}}, status=201)

    def _allowed(self, user: str, groups, ra: dict) -> bool:
        res = ra.get("resource", "") + (f"/{ra['subresource']}" if ra.get("subresource") else "")
        who = {user} | {f"group:{g}" for g in groups}
        return any(r["subject"] in who and ra.get("verb") in r["verbs"]
                   and r["resource"] == res
                   and ("*" in r["namespaces"] or ra.get("namespace", "") in r["namespaces"])
                   for r in self.rbac)

    async def _h_ssar(self, req: web.Request) -> web.Response:
        """SelfSubjectAccessReview: the request's own bearer token is the subject (401 for an
        unknown token; ``serve_self_review = False`` answers 404, as an apiserver without
        the API would)."""
        await self._pre(req)
        if not self.serve_self_review:
            return web.json_response({"kind": "Status", "code": 404}, status=404)
        auth = req.headers.get("Authorization", "")
        user = self.tokens.get(auth[7:] if auth.startswith("Bearer ") else "")
        if user is None:
            return web.json_response({"kind": "Status", "code": 401}, status=401)
        body = await req.json()
        ra = body.get("spec", {}).get("resourceAttributes", {})
        self.ssar_count += 1
        return web.json_response({**body, "status": {
            "allowed": self._allowed(user["username"], user["groups"], ra)}}, status=201)

    async def _h_event_create(self, req: web.Request) -> web.Response:
        await self._pre(req)
        ev = await req.json()
        ns = req.match_info["ns"]
        md = ev.setdefault("metadata", {})
        md["namespace"] = ns
        md.setdefault("name", md.pop("generateName", "event.") + uuid.uuid4().hex[:10])
        self.rv += 1
        md["resourceVersion"] = str(self.rv)
        self.k8s_events.append(ev)
        if len(self.k8s_events) > self.EVENTS_KEPT:     # as the apiserver's event TTL would
            del self.k8s_events[: len(self.k8s_events) - self.EVENTS_KEPT]
        return web.json_response(ev, status=201)

    async def _h_event_list(self, req: web.Request) -> web.Response:
        await self._pre(req)
        ns = req.match_info["ns"]
        items = [e for e in self.k8s_events if e["metadata"]["namespace"] == ns]
        return web.json_response({"kind": "EventList", "items": items})

    def events_for(self, ns: str, pod: str) -> List[dict]:
        return [e for e in self.k8s_events if e["metadata"]["namespace"] == ns
                and e.get("involvedObject", {}).get("name") == pod]

    async def _h_quota_list(self, req: web.Request):
        await self._pre(req)
        ns = req.match_info.get("ns", "")
        if req.query.get("watch") in ("true", "1"):
            return await self._watch(
                req, ns, _parse_selector(req.query.get("labelSelector", "")), [],
                history=self.quota_events, watchers=self.quota_watchers,
                current=lambda: [self._quota_view(q) for q in self.quotas.values()],
                kind="ResourceQuota")
        items = [self._quota_view(q) for (qns, _), q in self.quotas.items()
                 if not ns or qns == ns]
        return web.json_response({"kind": "ResourceQuotaList",
                                  "metadata": {"resourceVersion": str(self.rv)},
                                  "items": items})

    async def _h_pc_get(self, req: web.Request) -> web.Response:
        await self._pre(req)
        pc = self.priority_classes.get(req.match_info["name"])
        if pc is None:
            return web.json_response(
                {"kind": "Status", "status": "Failure", "reason": "NotFound", "code": 404,
                 "message": f'priorityclasses.scheduling.k8s.io "{req.match_info["name"]}" '
                            "not found"}, status=404)
        return web.json_response(pc)

    async def _h_pc_create(self, req: web.Request) -> web.Response:
        await self._pre(req)
        body = await req.json()
        name = (body.get("metadata") or {}).get("name", "")
        if not name or "value" not in body:
            return web.json_response({"kind": "Status", "code": 422, "reason": "Invalid",
                                      "message": "name and value are required"}, status=422)
        if name in self.priority_classes:
            return web.json_response({"kind": "Status", "code": 409, "reason": "AlreadyExists",
                                      "message": f'priorityclasses "{name}" already exists'},
                                     status=409)
        return web.json_response(self.apply_priority_classes(
            [dict(body, kind="PriorityClass")]) and self.priority_classes[name], status=201)

    async def _h_pc_list(self, req: web.Request) -> web.Response:
        await self._pre(req)
        return web.json_response({"kind": "PriorityClassList",
                                  "apiVersion": "scheduling.k8s.io/v1",
                                  "items": list(self.priority_classes.values())})

    async def _h_nodes(self, req: web.Request) -> web.Response:
        await self._pre(req)
        items = [{"metadata": {"name": n.name, "labels": n.labels},
                  "status": {"capacity": {n.resource: str(n.capacity)},
                             "allocatable": {n.resource: str(n.capacity)}}}
                 for n in self.nodes.values()]
        return web.json_response({"kind": "NodeList", "items": items})

    # ------------------------------------------------------------------------ audits
    def placeholders(self) -> List[dict]:
        return [p for p in self.pods.values()
                if (p["metadata"].get("labels") or {}).get("app") == "gpu-pool"]
