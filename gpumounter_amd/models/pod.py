"""Helpers over Kubernetes Pod JSON (plain dicts as returned by the REST API).

* :func:`qos_class` — kubelet's QoS classifier. The reference embeds a copy of it to compute the
  cgroup path (reference: pkg/util/cgroup/cgroup.go:171-237); this is an independent
  implementation of the documented rules (Guaranteed iff every container sets cpu+memory limits and
  requests equal limits; BestEffort iff nothing is set; else Burstable).
* :func:`parse_container_id` — handles ``docker://``, ``containerd://``, ``cri-o://`` (the
  reference strips only ``docker://``, util.go:23 — SURVEY defect 8).
* :func:`running_containers` — every running container, not just ``ContainerStatuses[0]``.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

_QTY = re.compile(r"^([+-]?[0-9.]+)([eE][+-]?[0-9]+)?(m|k|M|G|T|P|E|Ki|Mi|Gi|Ti|Pi|Ei)?$")
_SUFFIX = {
    None: Fraction(1), "m": Fraction(1, 1000), "k": Fraction(10**3), "M": Fraction(10**6),
    "G": Fraction(10**9), "T": Fraction(10**12), "P": Fraction(10**15), "E": Fraction(10**18),
    "Ki": Fraction(2**10), "Mi": Fraction(2**20), "Gi": Fraction(2**30), "Ti": Fraction(2**40),
    "Pi": Fraction(2**50), "Ei": Fraction(2**60),
}

QOS_GUARANTEED = "Guaranteed"
QOS_BURSTABLE = "Burstable"
QOS_BESTEFFORT = "BestEffort"
_QOS_RESOURCES = ("cpu", "memory")


def parse_quantity(q) -> Fraction:
    if isinstance(q, (int, float)):
        return Fraction(q)
    m = _QTY.match(str(q).strip())
    if not m:
        raise ValueError(f"bad quantity {q!r}")
    num = Fraction(m.group(1))
    if m.group(2):
        num *= Fraction(10) ** int(m.group(2)[1:])
    return num * _SUFFIX[m.group(3)]


def qos_class(pod: dict) -> str:
    if pod.get("status", {}).get("qosClass"):
        return pod["status"]["qosClass"]
    requests: Dict[str, Fraction] = {}
    limits: Dict[str, Fraction] = {}
    guaranteed = True
    containers = list(pod.get("spec", {}).get("containers", []))
    for c in containers:
        res = c.get("resources", {}) or {}
        for name, qty in (res.get("requests") or {}).items():
            if name in _QOS_RESOURCES:
                v = parse_quantity(qty)
                if v > 0:
                    requests[name] = requests.get(name, Fraction(0)) + v
        found = set()
        for name, qty in (res.get("limits") or {}).items():
            if name in _QOS_RESOURCES:
                v = parse_quantity(qty)
                if v > 0:
                    found.add(name)
                    limits[name] = limits.get(name, Fraction(0)) + v
        if not set(_QOS_RESOURCES) <= found:
            guaranteed = False
    if not requests and not limits:
        return QOS_BESTEFFORT
    if guaranteed:
        for name, req in requests.items():
            if limits.get(name) != req:
                guaranteed = False
                break
    if guaranteed and len(requests) == len(limits):
        return QOS_GUARANTEED
    return QOS_BURSTABLE


@dataclass(frozen=True)
class ContainerRef:
    name: str
    runtime: str          # docker | containerd | cri-o | ""
    id: str               # bare hex id
    running: bool
    # securityContext.privileged: the runtime already gave it every host device ("a *:* rwm"
    # and a /dev populated from the host), so gpumounter neither grants nor revokes anything there
    privileged: bool = False


def parse_container_id(cid: str) -> Tuple[str, str]:
    if not cid:
        return "", ""
    if "://" in cid:
        rt, _, bare = cid.partition("://")
        return rt, bare
    return "", cid


def privileged_containers(pod: dict) -> set:
    """Names of the pod's containers that run privileged."""
    return {c.get("name", "") for c in pod.get("spec", {}).get("containers", []) or []
            if ((c.get("securityContext") or {}).get("privileged") is True)}


def running_containers(pod: dict, only: str = "") -> List[ContainerRef]:
    out = []
    priv = privileged_containers(pod)
    for cs in pod.get("status", {}).get("containerStatuses", []) or []:
        if only and cs.get("name") != only:
            continue
        rt, bare = parse_container_id(cs.get("containerID", ""))
        running = "running" in (cs.get("state") or {})
        if bare:
            name = cs.get("name", "")
            out.append(ContainerRef(name, rt, bare, running, name in priv))
    return out


def meta(pod: dict) -> dict:
    return pod.get("metadata", {})


def name_of(pod: dict) -> str:
    return meta(pod).get("name", "")


def ns_of(pod: dict) -> str:
    return meta(pod).get("namespace", "")


def uid_of(pod: dict) -> str:
    return meta(pod).get("uid", "")


def node_of(pod: dict) -> str:
    return pod.get("spec", {}).get("nodeName", "") or ""


def phase_of(pod: dict) -> str:
    return pod.get("status", {}).get("phase", "")


def is_unschedulable(pod: dict) -> Optional[str]:
    """Return the scheduler message if the pod is marked Unschedulable (reference
    allocator.go:266 checks only Conditions[0]; here any PodScheduled=False condition counts)."""
    for cond in pod.get("status", {}).get("conditions", []) or []:
        if cond.get("type") == "PodScheduled" and cond.get("status") == "False" and \
                cond.get("reason") == "Unschedulable":
            return cond.get("message", "Unschedulable")
    return None


def is_terminating(pod: dict) -> bool:
    return bool(meta(pod).get("deletionTimestamp"))


def priority_of(pod: dict) -> int:
    """``spec.priority`` as the Priority admission plugin resolved it (0 when absent)."""
    try:
        return int(pod.get("spec", {}).get("priority") or 0)
    except (TypeError, ValueError):
        return 0


def nominated_node(pod: dict) -> str:
    """The node the scheduler reserved for a Pod whose preemption is under way."""
    return pod.get("status", {}).get("nominatedNodeName", "") or ""


def resource_limit(pod: dict, resource: str) -> int:
    total = 0
    for c in pod.get("spec", {}).get("containers", []) or []:
        lim = ((c.get("resources") or {}).get("limits") or {}).get(resource)
        if lim is not None:
            total += int(parse_quantity(lim))
    return total


def jcopy(x):
    """Deep copy of a JSON-shaped object (dicts, lists, scalars) — several times faster than
    copy.deepcopy, which pays for memo bookkeeping and arbitrary types."""
    t = type(x)
    if t is dict:
        return {k: jcopy(v) for k, v in x.items()}
    if t is list:
        return [jcopy(v) for v in x]
    return x


_DNS1123_LABEL = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?")
_DNS1123_SUBDOMAIN = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")


def is_dns1123_label(s: str) -> bool:
    """A namespace name (Kubernetes ``IsDNS1123Label``: ≤ 63 chars of [a-z0-9-])."""
    return len(s) <= 63 and bool(_DNS1123_LABEL.fullmatch(s))


def is_dns1123_subdomain(s: str) -> bool:
    """A Pod or node name (``IsDNS1123Subdomain``: ≤ 253 chars, dot-separated labels)."""
    return len(s) <= 253 and bool(_DNS1123_SUBDOMAIN.fullmatch(s))


def name_error(ns: str, name: str) -> Optional[str]:
    """Why ``ns``/``name`` cannot name a Pod (None: they can). Such a request is refused
    before anything else looks at it: no name the apiserver would refuse reaches a URL."""
    if not is_dns1123_label(ns):
        return f"Invalid param namespace: {ns!r}(must be a DNS-1123 label)"
    if not is_dns1123_subdomain(name):
        return f"Invalid param pod: {name!r}(must be a DNS-1123 subdomain)"
    return None
