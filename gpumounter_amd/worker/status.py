"""Worker node status: GPUs, ledger owners, placeholders, topology, per-namespace gauges.

The reference has no status endpoint; its collector only marks GPUs ALLOCATED from the kubelet's
PodResources ``List`` (reference: pkg/util/gpu/collector/collector.go:90-138). Here the same join
(device ID → GPU) feeds the NodeStatus RPC, the master's ``/api/v1/nodes/{node}/gpus`` and
``/api/v1/namespaces/{ns}/pods/{pod}/gpus``, and the ``gm_ledger_gpus``/``gm_hot_gpus`` gauges.
"""
from __future__ import annotations

import asyncio
from typing import Dict

from gpumounter_amd.hw import topology
from gpumounter_amd.models.device import gpus_by_key, normalize_device_id
from gpumounter_amd.models.types import ANN_CANDIDATE
from gpumounter_amd.node.ledger import LedgerError
from gpumounter_amd.node.procs import host_pid_ns
from gpumounter_amd.utils import log
from gpumounter_amd.worker.lease import expires_of

_log = log.get("worker.status")


async def node_status(svc, include_processes: bool) -> dict:
    """The node's GPUs, their ledger owners, the placeholders and the topology (the worker's
    NodeStatus RPC and ``/status``); refreshes the ledger and per-namespace gauges."""
    gpus = svc.inv.gpus()
    try:
        ledger = await svc.ledger.list()
    except LedgerError as e:
        ledger = []
        _log.error("ledger: %s", e)
    keys = gpus_by_key(gpus)
    for a in ledger:
        for d in a.device_ids:
            g = keys.get(normalize_device_id(d))
            if g is not None:
                g.pod_name, g.namespace, g.container = a.pod, a.namespace, a.container
                g.state = g.state.ALLOCATED
    phs = []
    for p in svc.ph.informer.list(lambda p: not p["metadata"].get("deletionTimestamp")):
        md = p["metadata"]
        ann = md.get("annotations") or {}
        ids = next((a.device_ids for a in ledger
                    if (a.namespace, a.pod) == (md["namespace"], md["name"])), ())
        phs.append({"namespace": md["namespace"], "name": md["name"],
                    "owner": ann.get("gpumounter.amd.com/owner-name", ""),
                    "owner_namespace": (md.get("labels") or {}).get(
                        "gpumounter.amd.com/owner-namespace", ""),
                    "owner_uid": ann.get("gpumounter.amd.com/owner-uid", ""),
                    "mode": ann.get("gpumounter.amd.com/mount-mode", ""),
                    # a ?lease= attach's end (Unix seconds), None without a lease
                    "lease_expires": expires_of(p),
                    # not the owner's GPUs (the owner's ledger view, WorkerService.pod_state,
                    # leaves them out): an unconfirmed trim/correction candidate, a failed
                    # attach's leftover the follow-up is deleting, a drained one
                    "releasing": ANN_CANDIDATE in ann or svc.is_abandoned(p) or
                                 md.get("uid") in svc.drain.unmarked,
                    "device_ids": list(ids)})
    out = {"node": svc.cfg.node_name,
           "gpus": [dict(g.to_dict(), healthy=g.index not in svc.unhealthy) for g in gpus],
           "placeholders": phs,
           "topology": topology.describe(gpus, svc.inv.links()),
           "ledger_api": svc.ledger.api_version, "kfd_major": svc.inv.kfd_major}
    if include_processes:
        def procs():
            by = {}
            for g in gpus:
                try:
                    by[g.index] = [p.__dict__ for p in svc.inv.processes(g.index)]
                except Exception as e:  # noqa: BLE001
                    by[g.index] = str(e)
            return by
        out["processes"] = await asyncio.to_thread(procs)     # amdsmi: off the loop
        # those PIDs are host-namespace numbers: comparable with this worker's only with hostPID
        out["host_pid_ns"] = host_pid_ns()
    for state in ("GPU_FREE_STATE", "GPU_ALLOCATED_STATE"):
        svc.metrics.ledger_gpus.labels(state=state).set(
            sum(1 for g in gpus if g.state.value == state))
    # hot-mounted GPUs per tenant namespace (chargeback: integrate over time in Prometheus)
    per_ns: Dict[str, int] = {}
    for ph in phs:
        if ph["mode"] != "standby" and ph["owner_namespace"] and not ph["releasing"]:
            per_ns[ph["owner_namespace"]] = per_ns.get(ph["owner_namespace"], 0) + \
                len(ph["device_ids"])
    for ns in set(svc._ns_seen) - set(per_ns):
        svc.metrics.hot_gpus.labels(namespace=ns).set(0)
    for ns, n in per_ns.items():
        svc.metrics.hot_gpus.labels(namespace=ns).set(n)
    svc._ns_seen = set(per_ns) | set(svc._ns_seen)
    return out
