"""Namespace GPU quotas for hot-mounted GPUs.

Kubernetes charges a pod's ``amd.com/gpu`` request against its namespace's ResourceQuota
(``requests.amd.com/gpu``). Placeholders in the shared pool namespace (the default,
``placeholder_namespace_mode=pool``) are charged to that pool namespace instead, so without a
check a tenant could hot-mount past the quota its administrator set. The reference has the same
hole: its slave pods always live in ``gpu-pool`` (reference:
pkg/util/gpu/allocator/allocator.go:189-234).

Here an attach into namespace N is refused when, for any ResourceQuota of N that limits the GPU
resource, ``used by N's own pods + GPUs hot-mounted into N's pods + requested > hard``. The
quota's ``status.used`` (kept by the quota controller) gives the first term; the second is read
from the placeholder labels in the pool namespace. In ``tenant`` placeholder mode the placeholders
live in N itself, so the apiserver's own quota admission already enforces it and nothing is added.

Quotas come from a list+watch of ResourceQuotas (:class:`~gpumounter_amd.cluster.informer.
QuotaInformer`, set by the worker): an attach into a namespace without a GPU quota makes no
apiserver call for it. Until that watch has synced (or without it) they are read through a short
TTL cache (a quota change applies within ``ttl_s``; the quota controller itself is asynchronous). Concurrent attaches into one namespace on one node are
serialised; across nodes, :meth:`GpuQuota.recheck` after the placeholders exist catches an
overshoot and rolls the attach back (two racing attaches may then both be refused, never both
admitted past the quota).
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass
from typing import Dict, List, Tuple

from gpumounter_amd.cluster.kube import ApiError, KubeClient
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.types import ANN_MOUNT_MODE, LABEL_OWNER_NS, MODE_STANDBY
from gpumounter_amd.utils import log

_log = log.get("cluster.quota")


DEVICECLASS_QUOTA_SUFFIX = ".deviceclass.resource.k8s.io/devices"


class QuotaExceeded(RuntimeError):
    pass


def _qty(v) -> int:
    """Integer GPU count from a quantity string ("4", "4000m" is not a valid GPU count)."""
    try:
        s = str(v).strip()
        if s.endswith("m"):
            return int(s[:-1]) // 1000
        return int(float(s))
    except (TypeError, ValueError):
        return 0


@dataclass
class Limit:
    quota: str
    key: str
    hard: int
    used_own: int


class GpuQuota:
    def __init__(self, cfg, kube: KubeClient, ttl_s: float = 2.0) -> None:
        self.cfg = cfg
        self.kube = kube
        self.ttl_s = ttl_s
        self.keys = (f"requests.{cfg.resource_name}", cfg.resource_name)
        if getattr(cfg, "gpu_allocation", "device-plugin") == "dra":
            # DRA: devices requested by the namespace's claims of the GPU device class
            self.keys = (f"{cfg.dra_device_class}{DEVICECLASS_QUOTA_SUFFIX}",)
        self._cache: Dict[str, Tuple[float, List[Limit]]] = {}
        self.informer = None     # QuotaInformer (Worker.start), else the TTL cache
        self._locks: Dict[str, asyncio.Lock] = {}
        self.checks = 0
        self.refusals = 0

    @property
    def active(self) -> bool:
        return self.cfg.quota_mode == "enforce" and self.cfg.placeholder_namespace_mode == "pool"

    def lock(self, ns: str) -> asyncio.Lock:
        lk = self._locks.get(ns)
        if lk is None:
            lk = self._locks[ns] = asyncio.Lock()
        return lk

    async def limits(self, ns: str) -> List[Limit]:
        inf = self.informer
        if inf is not None and inf._synced is not None and inf._synced.is_set():  # noqa: SLF001
            return self._limits(q for (qns, _), q in list(inf.cache.items()) if qns == ns)
        now = time.monotonic()
        hit = self._cache.get(ns)
        if hit is not None and now - hit[0] < self.ttl_s:
            return hit[1]
        try:
            items = await self.kube.list_resource_quotas(ns)
        except ApiError as e:
            if e.status == 404:
                items = []
            else:
                raise
        out = self._limits(items)
        self._cache[ns] = (now, out)
        return out

    def _limits(self, items) -> List[Limit]:
        out: List[Limit] = []
        for q in items:
            hard = (q.get("spec") or {}).get("hard") or {}
            used = (q.get("status") or {}).get("used") or {}
            for k in self.keys:
                if k in hard:
                    out.append(Limit(q["metadata"]["name"], k, _qty(hard[k]), _qty(used.get(k, 0))))
                    break
        return out

    async def hot_in_namespace(self, ns: str) -> int:
        """GPUs held by pool placeholders whose owner pod lives in ``ns``."""
        sel = f"{LABEL_OWNER_NS}={ns}"
        pods, _ = await self.kube.list_pods(self.cfg.pool_namespace, label_selector=sel)
        total = 0
        for p in pods:
            md = p["metadata"]
            if md.get("deletionTimestamp") or \
                    (md.get("annotations") or {}).get(ANN_MOUNT_MODE) == MODE_STANDBY:
                continue
            gpus = (md.get("annotations") or {}).get("gpumounter.amd.com/gpus")
            total += int(gpus) if gpus and gpus.isdigit() else \
                podu.resource_limit(p, self.cfg.resource_name)
        return total

    async def check(self, ns: str, n: int, already_counted: int = 0) -> None:
        """Raise :class:`QuotaExceeded` if ``n`` more GPUs would exceed a quota of ``ns``.
        ``already_counted``: GPUs of this attach that the placeholder list already contains
        (the post-create recheck)."""
        if not self.active or n <= 0:
            return
        self.checks += 1
        lims = await self.limits(ns)
        if not lims:
            return
        hot = await self.hot_in_namespace(ns) - already_counted
        for lim in lims:
            if lim.used_own + hot + n > lim.hard:
                self.refusals += 1
                raise QuotaExceeded(
                    f"exceeded quota: {lim.quota}, requested: {lim.key}={n}, used: "
                    f"{lim.key}={lim.used_own + hot} ({lim.used_own} by pods, {hot} hot-mounted), "
                    f"limited: {lim.key}={lim.hard}")

    async def recheck(self, ns: str, n: int) -> None:
        """After this attach's placeholders exist: did a concurrent attach elsewhere overshoot?"""
        await self.check(ns, n, already_counted=n)
