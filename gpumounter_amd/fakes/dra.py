"""Dynamic Resource Allocation (``resource.k8s.io/v1``) for the hermetic apiserver.

Clusters whose GPUs are published by a DRA driver have no ``amd.com/gpu`` extended resource:
a Pod asks for devices through a ResourceClaim, the scheduler allocates devices of the node's
ResourceSlices to the claim (``status.allocation``) before it binds the Pod, and the claim
records which Pods use it (``status.reservedFor``). This module models that much:

* one ResourceSlice per DRA node (driver ``gpu.amd.com``, pool = node name), one device per GPU
  (``gpu-<index>``) with attributes ``pciAddr``, ``uuid``, ``index``, ``productName``;
* ResourceClaim create/get/list/watch/delete (watch events share the Pods' resourceVersion
  sequence; quota admission for ``<class>.deviceclass.resource.k8s.io/devices``), with device
  requests of ``exactly`` count N from a
  device class, optionally narrowed by CEL selectors of the forms
  ``device.attributes["<driver>"].pciAddr in ["…", …]`` and ``… == "…"`` (others are refused
  at create, so a test cannot silently rely on unsupported CEL);
* scheduling of Pods that reference claims by ``resourceClaimName``: all of the Pod's claims
  are allocated on one node or the Pod is Unschedulable; an allocated claim is reused; the
  claims' status (allocation, reservedFor) is written before the Pod is bound;
* deallocation when no Pod holds the claim any more, and when it is deleted.

Parity with a real scheduler and with the AMD DRA driver's attribute names is unpinned (no
cluster here); the worker reads the BDF attribute name from config (``dra_bdf_attribute``).
"""
from __future__ import annotations

import json
import re
import uuid
from typing import Dict, List, Optional, Tuple

from aiohttp import web

from gpumounter_amd.models import pod as podu

DRIVER = "gpu.amd.com"
API = "resource.k8s.io/v1"
_IN = re.compile(r'^\s*device\.attributes\["([^"]+)"\]\.(\w+)\s+in\s+\[(.*)\]\s*$', re.S)
_EQ = re.compile(r'^\s*device\.attributes\["([^"]+)"\]\.(\w+)\s*==\s*"([^"]*)"\s*$')
_STR = re.compile(r'"([^"]*)"')


def parse_selector(expr: str) -> Tuple[str, str, List[str]]:
    """(domain, attribute, allowed values) of a supported CEL selector; ValueError otherwise."""
    m = _IN.match(expr)
    if m:
        return m.group(1), m.group(2), _STR.findall(m.group(3))
    m = _EQ.match(expr)
    if m:
        return m.group(1), m.group(2), [m.group(3)]
    raise ValueError(f"unsupported CEL selector: {expr!r}")


class DraState:
    """Claims and device allocation; owned by the FakeCluster (its ``dra`` attribute)."""

    HISTORY = 4096

    def __init__(self, cluster) -> None:
        self.cluster = cluster
        self.claims: Dict[Tuple[str, str], dict] = {}
        self.events: List[tuple] = []          # watch history: (rv, type, snapshot)
        self.watchers: List[tuple] = []

    def _bump(self, etype: str, claim: dict) -> None:
        self.cluster.rv += 1
        claim["metadata"]["resourceVersion"] = str(self.cluster.rv)
        data = json.dumps(claim).encode()        # serialized: see FakeCluster._bump
        self.events.append((self.cluster.rv, etype, data))
        if len(self.events) > self.HISTORY:
            del self.events[: len(self.events) - self.HISTORY]
        for q, ns, lsel, fsel in list(self.watchers):
            if self.cluster._matches(claim, ns, lsel, fsel):   # noqa: SLF001
                q.put_nowait((etype, data))
        self.cluster.quota_touch(claim["metadata"].get("namespace", ""))

    # ------------------------------------------------------------------------ slices
    def slices(self, node_name: str = "") -> List[dict]:
        out = []
        for n in self.cluster.nodes.values():
            if getattr(n, "gpu_api", "device-plugin") != "dra":
                continue
            if node_name and n.name != node_name:
                continue
            out.append({"apiVersion": API, "kind": "ResourceSlice",
                        "metadata": {"name": f"{n.name}-{DRIVER}"},
                        "spec": {"driver": DRIVER, "nodeName": n.name,
                                 "pool": {"name": n.name, "generation": 1,
                                          "resourceSliceCount": 1},
                                 "devices": [self.device(g) for g in n.gpus]}})
        return out

    @staticmethod
    def device(g) -> dict:
        return {"name": f"gpu-{g.index}",
                "attributes": {"pciAddr": {"string": g.bdf}, "uuid": {"string": g.uuid},
                               "index": {"int": g.index},
                               "productName": {"string": "AMD Instinct MI355X"}}}

    # ------------------------------------------------------------------------ claims
    def create(self, ns: str, body: dict) -> dict:
        claim = podu.jcopy(body)
        md = claim.setdefault("metadata", {})
        name = md.get("name", "")
        if not name:
            raise web.HTTPUnprocessableEntity(text=json.dumps(
                {"kind": "Status", "message": "name is required"}))
        if (ns, name) in self.claims:
            raise web.HTTPConflict(text=json.dumps(
                {"kind": "Status", "reason": "AlreadyExists",
                 "message": f'resourceclaims "{name}" already exists'}),
                content_type="application/json")
        for r in (claim.get("spec", {}).get("devices", {}).get("requests") or []):
            for s in (r.get("exactly") or {}).get("selectors") or []:
                try:
                    parse_selector((s.get("cel") or {}).get("expression", ""))
                except ValueError as e:
                    raise web.HTTPUnprocessableEntity(text=json.dumps(
                        {"kind": "Status", "message": str(e)}),
                        content_type="application/json") from e
        self._quota_admit(ns, claim)
        md["namespace"] = ns
        md["uid"] = str(uuid.uuid4())
        claim["status"] = {}
        self.claims[(ns, name)] = claim
        self._bump("ADDED", claim)
        # Pods waiting for this claim can be scheduled now
        for key in list(self.cluster._unschedulable):   # noqa: SLF001
            self.cluster._spawn(self.cluster._schedule(*key))   # noqa: SLF001
        return claim

    @staticmethod
    def _requested(claim: dict, device_class: str) -> int:
        return sum(int((r.get("exactly") or {}).get("count", 1))
                   for r in (claim.get("spec", {}).get("devices", {}).get("requests") or [])
                   if (r.get("exactly") or {}).get("deviceClassName") == device_class)

    def quota_used(self, ns: str, device_class: str) -> int:
        """``<class>.deviceclass.resource.k8s.io/devices`` usage: devices the namespace's
        claims request from that class."""
        return sum(self._requested(c, device_class) for (cns, _), c in self.claims.items()
                   if cns == ns)

    def _quota_admit(self, ns: str, claim: dict) -> None:
        from gpumounter_amd.fakes.apiserver import DEVICECLASS_QUOTA_SUFFIX

        for (qns, qname), q in self.cluster.quotas.items():
            if qns != ns:
                continue
            for key, hard in q["spec"]["hard"].items():
                if not key.endswith(DEVICECLASS_QUOTA_SUFFIX):
                    continue
                dc = key[:-len(DEVICECLASS_QUOTA_SUFFIX)]
                want = self._requested(claim, dc)
                used = self.quota_used(ns, dc)
                if want and used + want > int(hard):
                    raise web.HTTPForbidden(text=json.dumps(
                        {"kind": "Status", "reason": "Forbidden", "code": 403,
                         "message": f'resourceclaims "{claim["metadata"].get("name")}" is '
                                    f"forbidden: exceeded quota: {qname}, requested: "
                                    f"{key}={want}, used: {key}={used}, limited: {key}={hard}"}),
                        content_type="application/json")

    def delete(self, ns: str, name: str) -> Optional[dict]:
        claim = self.claims.pop((ns, name), None)
        if claim is not None:
            self._deallocate(ns, claim, bump=False)
            self._bump("DELETED", claim)
        return claim

    def _deallocate(self, ns: str, claim: dict, bump: bool = True) -> None:
        if claim.get("status", {}).get("allocation"):
            for n in self.cluster.nodes.values():
                n.release_pod(ns, "claim:" + claim["metadata"]["name"])
            claim["status"].pop("allocation", None)
            if bump:
                self._bump("MODIFIED", claim)
            freed = True
        else:
            freed = False
        if freed:   # capacity freed: retry unschedulable pods (scheduler queue)
            for key in list(self.cluster._unschedulable):   # noqa: SLF001
                self.cluster._spawn(self.cluster._schedule(*key))   # noqa: SLF001

    def refs(self, pod: dict) -> List[str]:
        return [c.get("resourceClaimName", "") for c in
                (pod.get("spec", {}).get("resourceClaims") or [])]

    # ------------------------------------------------------------------------ scheduling
    def schedule(self, pod: dict, candidates) -> Tuple[Optional[str], str]:
        """Allocate the Pod's claims on the first fitting node: (node name, "") or
        (None, why). Allocations made here are committed (claims reserved for the Pod)."""
        ns = podu.ns_of(pod)
        names = self.refs(pod)
        claims = []
        for cname in names:
            c = self.claims.get((ns, cname))
            if c is None:
                return None, f'waiting for resourceclaim "{cname}"'
            claims.append(c)
        for n in candidates:
            if getattr(n, "gpu_api", "device-plugin") != "dra":
                continue
            plan = self._plan(n, claims)
            if plan is None:
                continue
            for c, devs in zip(claims, plan):
                st = c.setdefault("status", {})
                if devs is not None:   # newly allocated on n
                    st["allocation"] = {"devices": {"results": [
                        {"request": req, "driver": DRIVER, "pool": n.name, "device": d}
                        for req, d in devs]},
                        "nodeSelector": {"nodeSelectorTerms": [{"matchFields": [
                            {"key": "metadata.name", "operator": "In", "values": [n.name]}]}]}}
                    ids = [n.device_id(g) for d in devs for g in n.gpus
                           if f"gpu-{g.index}" == d[1]]
                    n.record(ns, "claim:" + c["metadata"]["name"], "claim", ids,
                             uid=c["metadata"]["uid"])
                rf = st.setdefault("reservedFor", [])
                if not any(r.get("uid") == podu.uid_of(pod) for r in rf):
                    rf.append({"resource": "pods", "name": podu.name_of(pod),
                               "uid": podu.uid_of(pod)})
                # the scheduler writes the claim's status before it binds the Pod
                self._bump("MODIFIED", c)
            return n.name, ""
        return None, "cannot allocate all claims"

    def _plan(self, node, claims):
        """Per claim: None (already allocated on this node) or [(request, device)] to allocate;
        None overall if some claim does not fit."""
        taken = {d for c in self.claims.values()
                 for r in (c.get("status", {}).get("allocation") or {}).get("devices", {})
                 .get("results", []) if r.get("pool") == node.name for d in [r["device"]]}
        plan = []
        for c in claims:
            alloc = (c.get("status", {}).get("allocation") or {}).get("devices", {})
            if alloc:
                if any(r.get("pool") != node.name for r in alloc.get("results", [])):
                    return None
                plan.append(None)
                continue
            devs = []
            for r in (c.get("spec", {}).get("devices", {}).get("requests") or []):
                ex = r.get("exactly") or {}
                count = int(ex.get("count", 1))
                filters = []
                for s in ex.get("selectors") or []:
                    dom, attr, vals = parse_selector((s.get("cel") or {}).get("expression", ""))
                    filters.append((dom, attr, {v.lower() for v in vals}))
                free = [g for g in node.gpus if f"gpu-{g.index}" not in taken and
                        node.device_id(g) not in node.unhealthy and
                        all(dom == DRIVER and self._attr(g, attr) in vals
                            for dom, attr, vals in filters)]
                if len(free) < count:
                    return None
                for g in free[:count]:
                    devs.append((r.get("name", ""), f"gpu-{g.index}"))
                    taken.add(f"gpu-{g.index}")
            plan.append(devs)
        return plan

    @classmethod
    def _attr(cls, g, name: str) -> str:
        v = cls.device(g)["attributes"].get(name) or {}
        return str(next(iter(v.values()), "")).lower()

    def pod_gone(self, pod: dict) -> None:
        """A Pod left: drop it from its claims' reservedFor; a claim no Pod holds is
        deallocated (the resourceclaim controller's job)."""
        ns = podu.ns_of(pod)
        for cname in self.refs(pod):
            c = self.claims.get((ns, cname))
            if c is None:
                continue
            rf = [r for r in c.get("status", {}).get("reservedFor", [])
                  if r.get("uid") != podu.uid_of(pod)]
            c.setdefault("status", {})["reservedFor"] = rf
            if not rf and c["status"].get("allocation"):
                self._deallocate(ns, c)
            else:
                self._bump("MODIFIED", c)
        # claims owned by the Pod (ownerReferences) are garbage-collected with it
        for (cns, cname), c in list(self.claims.items()):
            if cns == ns and any(o.get("uid") == podu.uid_of(pod)
                                 for o in c["metadata"].get("ownerReferences") or []):
                self.delete(cns, cname)

    # ------------------------------------------------------------------------ HTTP
    def install(self, r: web.UrlDispatcher, pre) -> None:
        base = f"/apis/{API}"

        async def list_slices(req):
            await pre(req)
            node = ""
            for part in req.query.get("fieldSelector", "").split(","):
                k, _, v = part.partition("=")
                if k.strip() == "spec.nodeName":
                    node = v.strip()
            return web.json_response({"kind": "ResourceSliceList", "apiVersion": API,
                                      "items": self.slices(node)})

        async def list_claims(req):
            from gpumounter_amd.fakes.apiserver import _parse_selector

            await pre(req)
            ns = req.match_info.get("ns", "")
            lsel = _parse_selector(req.query.get("labelSelector", ""))
            if req.query.get("watch") in ("true", "1"):
                return await self.cluster._watch(   # noqa: SLF001
                    req, ns, lsel, [], history=self.events, watchers=self.watchers,
                    current=lambda: list(self.claims.values()), kind="ResourceClaim")
            items = [c for c in self.claims.values()
                     if self.cluster._matches(c, ns, lsel, [])]   # noqa: SLF001
            return web.json_response({"kind": "ResourceClaimList", "apiVersion": API,
                                      "metadata": {"resourceVersion": str(self.cluster.rv)},
                                      "items": items})

        async def create_claim(req):
            await pre(req)
            return web.json_response(self.create(req.match_info["ns"], await req.json()),
                                     status=201)

        async def get_claim(req):
            await pre(req)
            c = self.claims.get((req.match_info["ns"], req.match_info["name"]))
            if c is None:
                return web.json_response({"kind": "Status", "reason": "NotFound", "code": 404,
                                          "message": "resourceclaim not found"}, status=404)
            return web.json_response(c)

        async def delete_claim(req):
            await pre(req)
            c = self.delete(req.match_info["ns"], req.match_info["name"])
            if c is None:
                return web.json_response({"kind": "Status", "reason": "NotFound", "code": 404,
                                          "message": "resourceclaim not found"}, status=404)
            return web.json_response(c)

        r.add_get(f"{base}/resourceslices", list_slices)
        r.add_get(f"{base}/resourceclaims", list_claims)
        r.add_get(f"{base}/namespaces/{{ns}}/resourceclaims", list_claims)
        r.add_post(f"{base}/namespaces/{{ns}}/resourceclaims", create_claim)
        r.add_get(f"{base}/namespaces/{{ns}}/resourceclaims/{{name}}", get_claim)
        r.add_delete(f"{base}/namespaces/{{ns}}/resourceclaims/{{name}}", delete_claim)
