"""The node's GPU ledger on clusters that allocate GPUs with DRA (``resource.k8s.io/v1``).

With a DRA driver there is no ``amd.com/gpu`` extended resource, so the device manager (its
checkpoint, PodResources ``devices``) knows nothing about GPUs. What the scheduler allocated is
in the ResourceClaims instead: ``status.allocation.devices.results`` names (driver, pool,
device), and ``status.reservedFor`` the Pods holding the claim. The device's PCI address comes
from the node's ResourceSlice (attribute ``dra_bdf_attribute``, or any attribute whose value is
a PCI address). :class:`DraLedger` serves the same interface as
:class:`~gpumounter_amd.node.ledger.LedgerClient` (``get``, ``list``, ``by_pod``,
``allocatable``), so placeholders, admission, audits and the reconciler work unchanged.

The reference only knows the device-plugin model (reference:
pkg/util/gpu/collector/collector.go:90-138 reads PodResources ``devices``).
"""
from __future__ import annotations

import re
import time
from typing import Callable, Dict, List, Optional, Tuple

from gpumounter_amd.cluster.kube import ApiError, NotFound
from gpumounter_amd.node.ledger import Allocation, LedgerError
from gpumounter_amd.utils import log

_log = log.get("node.dra")
_BDF = re.compile(r"^[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-7]$")


def claim_names(pod: dict) -> List[str]:
    """ResourceClaims a Pod uses: named ones, and the ones generated from templates (their
    names are in status.resourceClaimStatuses)."""
    out = [c.get("resourceClaimName") for c in (pod.get("spec", {}).get("resourceClaims") or [])
           if c.get("resourceClaimName")]
    out += [s.get("resourceClaimName") for s in
            (pod.get("status", {}).get("resourceClaimStatuses") or [])
            if s.get("resourceClaimName") and s.get("resourceClaimName") not in out]
    return out


class DraLedger:
    SLICE_TTL_S = 30.0

    def __init__(self, kube, node: str, driver: str, device_class: str, bdf_attribute: str,
                 pod_lookup: Optional[Callable[[str, str], Optional[dict]]] = None) -> None:
        self.kube = kube
        self.node = node
        self.driver = driver
        self.device_class = device_class
        self.bdf_attribute = bdf_attribute
        self.pod_lookup = pod_lookup
        self._dev: Dict[Tuple[str, str], str] = {}    # (pool, device name) → BDF
        self._dev_at = 0.0
        # ClaimInformer over the placeholders' claims (set by the worker): their allocation is
        # read from its cache; other claims (a tenant's own) with a GET
        self.claims = None
        self.claim_cache_hits = 0
        self.calls = 0
        self.throttled = 0

    @property
    def api_version(self) -> str:
        return "resource.k8s.io/v1"

    async def close(self) -> None:
        pass

    # ------------------------------------------------------------------------ slices
    def _bdf(self, attrs: dict) -> str:
        for key in (self.bdf_attribute, f"{self.driver}/{self.bdf_attribute}"):
            v = attrs.get(key)
            if isinstance(v, dict) and v:
                return str(next(iter(v.values())))
        for v in attrs.values():        # any attribute that is a PCI address
            s = next(iter(v.values()), "") if isinstance(v, dict) and v else ""
            if isinstance(s, str) and _BDF.match(s):
                return s
        return ""

    async def devices(self, refresh: bool = False) -> Dict[Tuple[str, str], str]:
        """(pool, device) → PCI BDF of this node's devices of our driver (cached)."""
        if refresh or not self._dev or time.monotonic() - self._dev_at > self.SLICE_TTL_S:
            self.calls += 1
            try:
                slices = await self.kube.list_slices(self.node)
            except ApiError as e:
                raise LedgerError(f"ResourceSlices of {self.node}: {e}") from e
            m: Dict[Tuple[str, str], str] = {}
            for sl in slices:
                spec = sl.get("spec", {})
                if spec.get("driver") != self.driver or spec.get("nodeName") not in (
                        None, "", self.node):
                    continue
                pool = (spec.get("pool") or {}).get("name", "")
                for d in spec.get("devices") or []:
                    bdf = self._bdf(d.get("attributes") or {})
                    if bdf:
                        m[(pool, d.get("name", ""))] = bdf
            self._dev, self._dev_at = m, time.monotonic()
        return self._dev

    async def claim_devices(self, claim: dict) -> List[str]:
        """BDFs of this node's devices allocated to the claim (driver ours)."""
        results = (((claim.get("status") or {}).get("allocation") or {}).get("devices") or {}
                   ).get("results") or []
        mine = [(r.get("pool", ""), r.get("device", "")) for r in results
                if r.get("driver") == self.driver]
        if not mine:
            return []
        devs = await self.devices()
        if any(k not in devs for k in mine):
            devs = await self.devices(refresh=True)       # a slice that changed meanwhile
        return [devs[k] for k in mine if k in devs]

    def reserved_devices(self, namespace: str, claim: str, pod_uid: str
                         ) -> Optional[Tuple[str, ...]]:
        """BDFs of a claim in the watch cache that is allocated and reserved for ``pod_uid``,
        without any request; None when the cache cannot tell. The scheduler writes both before
        it binds the Pod, and from then on the devices are the claim's in its books: the DRA
        counterpart of reading the device-manager checkpoint at admission."""
        c = self.claims.cache.get((namespace, claim)) if self.claims is not None else None
        if c is None:
            return None
        st = c.get("status") or {}
        if not any(r.get("uid") == pod_uid for r in st.get("reservedFor") or []):
            return None
        keys = [(r.get("pool", ""), r.get("device", "")) for r in
                ((st.get("allocation") or {}).get("devices") or {}).get("results") or []
                if r.get("driver") == self.driver]
        if not keys or any(k not in self._dev for k in keys):
            return None
        self.claim_cache_hits += 1
        return tuple(self._dev[k] for k in keys)

    # ------------------------------------------------------------------------ ledger API
    async def get(self, namespace: str, pod: str) -> Optional[List[str]]:
        p = self.pod_lookup(namespace, pod) if self.pod_lookup else None
        if p is None:
            try:
                p = await self.kube.get_pod(namespace, pod)
            except NotFound:
                return []
            except ApiError as e:
                raise LedgerError(f"pod {namespace}/{pod}: {e}") from e
        out: List[str] = []
        uid = p.get("metadata", {}).get("uid")

        def held(c: dict) -> bool:
            reserved = (c.get("status") or {}).get("reservedFor") or []
            return not (reserved and uid and not any(r.get("uid") == uid for r in reserved))

        for cname in claim_names(p):
            cached = self.claims.cache.get((namespace, cname)) if self.claims else None
            if cached is not None and held(cached) and \
                    (cached.get("status") or {}).get("allocation"):
                self.claim_cache_hits += 1
                out += await self.claim_devices(cached)
                continue
            self.calls += 1
            try:
                claim = await self.kube.get_claim(namespace, cname)
            except NotFound:
                continue
            except ApiError as e:
                raise LedgerError(f"resourceclaim {namespace}/{cname}: {e}") from e
            if not held(claim):
                continue       # allocated, but not (yet / any more) for this Pod
            out += await self.claim_devices(claim)
        return out

    async def list(self, resource_only: bool = True) -> List[Allocation]:
        self.calls += 1
        try:
            claims = await self.kube.list_claims()
        except ApiError as e:
            raise LedgerError(f"ResourceClaims: {e}") from e
        devs = await self.devices()
        out: List[Allocation] = []
        for c in claims:
            results = (((c.get("status") or {}).get("allocation") or {}).get("devices") or {}
                       ).get("results") or []
            keys = [(r.get("pool", ""), r.get("device", "")) for r in results
                    if r.get("driver") == self.driver]
            if not keys:
                continue
            if any(k not in devs for k in keys):
                devs = await self.devices(refresh=True)
            ids = tuple(devs[k] for k in keys if k in devs)
            if not ids:
                continue        # another node's devices
            ns = c["metadata"].get("namespace", "")
            for r in (c.get("status") or {}).get("reservedFor") or []:
                if r.get("resource", "pods") == "pods":
                    out.append(Allocation(ns, r.get("name", ""), "", self.device_class, ids))
        return out

    async def by_pod(self) -> Dict[Tuple[str, str], List[str]]:
        out: Dict[Tuple[str, str], List[str]] = {}
        for a in await self.list():
            out.setdefault((a.namespace, a.pod), []).extend(a.device_ids)
        return out

    async def allocatable(self) -> Optional[List[str]]:
        return sorted(set((await self.devices(refresh=True)).values()))
