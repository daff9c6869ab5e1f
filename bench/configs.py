"""BASELINE.json's named configurations as runnable scenarios (one JSON line each).

  scale       "scale one Pod 1→8 MI355X then back to 0 (xGMI-hive-aware attach order)":
              per-step attach/detach latency plus the topology of the attached set.
  contention  "4 Pods contending for 8 MI355X; k8s scheduler ledger stays consistent":
              concurrent rounds of adds/removes from 4 pods, invariant checks after each round.
  soak        "1000 attach/detach cycles across 8 GPUs; p99 latency + zero orphaned cgroup
              entries": cycles of 1-4 GPUs, single and entire mounts, final orphan audit.
  placement   placement quality on a fragmented node with a device plugin that ignores
              gpumounter's hint (the honest default of the fake): attaches compared with the
              best set the free GPUs allowed.
  chaos       contention with faults injected at every mutating worker stage and the worker
              SIGKILLed with requests in flight every few rounds (process deployment):
              invariants after every round, and how long the node took to converge.

The control plane is the hermetic fake (apiserver, scheduler, kubelet); node operations are the
production ones (cgroup rule backends, device-node writer) in their unprivileged modes. Runs
with the real libamd_smi when GPUs are present (``--amdsmi ""``) or the bundled 8×MI355X mock.
"""
from __future__ import annotations

import argparse
import asyncio
import contextlib
import json
import os
import random
import shutil
import subprocess
import sys
import time
from typing import Dict, List, Optional

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpumounter_amd.fakes.apiserver import LatencyModel  # noqa: E402
from gpumounter_amd.fakes.harness import LocalCluster  # noqa: E402
from gpumounter_amd.hw import topology  # noqa: E402
from gpumounter_amd.utils import log, runtime  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(int(q * len(xs)), len(xs) - 1)] if xs else None


def _real_dev_nodes(pid: int) -> list:
    """GPU-like device nodes (DRM major 226 or the KFD major) under a real tenant's /dev."""
    import stat
    out = []
    root = f"/proc/{pid}/root/dev"
    for dirpath, _, files in os.walk(root):
        for f in files:
            st = os.lstat(os.path.join(dirpath, f))
            if stat.S_ISCHR(st.st_mode) and os.major(st.st_rdev) in (226, 511):
                out.append(os.path.relpath(os.path.join(dirpath, f), root))
    return sorted(out)


def _tenant(lc, args, name: str) -> None:
    """A tenant pod; with --node-ops real its container is a real process in its own mount
    namespace (private tmpfs /dev) inside a real cgroup2 cgroup carrying a runc-style device
    program, so every attach loads/updates a real BPF program and mknods real nodes."""
    sb = getattr(args, "sandbox", None)
    if sb is None:
        lc.tenant(name)
        return
    from gpumounter_amd.fakes.realnode import attach_runtime_program
    pid = sb.spawn_tenant()
    lc.tenant(name, pids={"main": [pid]})
    (ctr,) = [c for c in lc.nodes["node-0"].node.containers.values() if c.pod_name == name]
    attach_runtime_program(ctr.cgroup_dir)
    args.tenant_pids[name] = pid


async def invariants(lc, tenants, why=None) -> int:
    """Number of violated ledger invariants (0 = consistent); ``why`` collects descriptions."""
    bad = 0
    why = why if why is not None else []
    node = lc.nodes["node-0"].node
    held = list(node.allocated)
    bad += len(held) != len(set(held))
    svc = lc.nodes["node-0"].worker.service
    hot = 0
    for t in tenants:
        pod = lc.cluster.get("default", t)
        st = await svc.pod_state(pod)
        hot += len(st.hot)
        issues = svc.hm.audit(pod, st.hot, st.own)
        bad += len(issues)
        if issues:
            why.append(f"{t}: audit {[(i.kind, i.path) for i in issues[:4]]}")
    # GPUs held by warm-pool standby placeholders (a standby the pool's refill created while
    # concurrent attaches filled the node stays Pending, holding nothing, until the pool drops it)
    standby_names = {p["metadata"]["name"] for p in lc.cluster.placeholders()
                     if (p["metadata"].get("annotations") or {}).get(
                         "gpumounter.amd.com/mount-mode") == "standby"}
    standby = sum(1 for _, pod, _ in node.allocated.values() if pod in standby_names)
    if hot + standby != len(node.allocated):
        bad += 1
        why.append(f"hot {hot} + standby {standby} != allocated {len(node.allocated)}: "
                   f"{sorted(set(pod for _, pod, _ in node.allocated.values()))}")
    bad += len(node.free_ids()) + len(node.allocated) != node.capacity
    return bad


async def scale(lc, args) -> dict:
    _tenant(lc, args, "scaler")
    inv = lc.inventory
    steps = []
    uuids = []
    n_gpus = len(lc.nodes["node-0"].node.gpus)
    for k in range(1, n_gpus + 1):
        t0 = time.perf_counter()
        code, b = await lc.add("default", "scaler", 1)
        ms = (time.perf_counter() - t0) * 1e3
        if code != 200:
            raise RuntimeError(f"attach #{k}: {code} {b}")
        uuids.append(b["devices"][0]["uuid"])
        svc = lc.nodes["node-0"].worker.service
        st = await svc.pod_state(lc.cluster.get("default", "scaler"))
        table = {g.index: g for g in st.hot}
        s, hives, numa, non_xgmi = topology.score_set(table, inv.links(), sorted(table))
        steps.append({"gpus": k, "attach_ms": round(ms, 3), "added": b["devices"][0]["bdf"],
                      "numa_nodes": numa, "hives": hives, "non_xgmi_pairs": non_xgmi})
    down = []
    for k, u in enumerate(reversed(uuids)):
        t0 = time.perf_counter()
        code, _ = await lc.remove("default", "scaler", [u])
        down.append(round((time.perf_counter() - t0) * 1e3, 3))
        if code != 200:
            raise RuntimeError(f"detach #{k}: {code}")
    # NUMA nodes may only be crossed once the first socket is full
    per_numa = {}
    for g in lc.nodes["node-0"].node.gpus:
        per_numa[g.numa_node] = per_numa.get(g.numa_node, 0) + 1
    first = max(per_numa.values())
    numa_ok = all(s["numa_nodes"] == 1 for s in steps[:first])
    return {"steps": steps, "detach_ms": down, "numa_packed": numa_ok,
            "audit_issues": len(await lc.audit("default", "scaler")),
            "placeholders_left": len(lc.cluster.placeholders())}


async def contention(lc, args) -> dict:
    tenants = [f"c{i}" for i in range(4)]
    for t in tenants:
        _tenant(lc, args, t)
    rnd = random.Random(args.seed)
    svc = lc.nodes["node-0"].worker.service
    ok = fail = 0
    lat = []
    violations = 0
    examples: list = []
    t_start = time.perf_counter()
    for _ in range(args.rounds):
        async def op(t):
            nonlocal ok, fail
            st = await svc.pod_state(lc.cluster.get("default", t))
            if st.hot and rnd.random() < 0.5:
                ids = [g.uuid for g in st.hot] if st.mount_type.value == "entire-mount" else \
                    [g.uuid for g in rnd.sample(st.hot, rnd.randint(1, len(st.hot)))]
                code, _ = await lc.remove("default", t, ids, force=True)
            else:
                t0 = time.perf_counter()
                code, _ = await lc.add("default", t, rnd.randint(1, 4),
                                       entire=rnd.random() < 0.3)
                if code == 200:
                    lat.append((time.perf_counter() - t0) * 1e3)
            if code == 200:
                ok += 1
            else:
                fail += 1
        await asyncio.gather(*[op(t) for t in tenants])
        why: list = []
        bad = await invariants(lc, tenants, why)
        if bad and getattr(args, "faults", False):
            # a failed operation's cleanup may be with the reconciler's follow-up (retried
            # after 0.1-5 s): the node must converge, not be consistent the instant ops return
            t0 = time.perf_counter()
            while bad and time.perf_counter() - t0 < 10:
                await asyncio.sleep(0.05)
                why = []
                bad = await invariants(lc, tenants, why)
        violations += bad
        examples.extend(why[:2])
    elapsed = time.perf_counter() - t_start
    return {"rounds": args.rounds, "ops_ok": ok, "ops_refused": fail,
            "ops_per_s": round((ok + fail) / elapsed, 1),
            "attach_p50_ms": round(pct(lat, 0.5), 3) if lat else None,
            "attach_p99_ms": round(pct(lat, 0.99), 3) if lat else None,
            "invariant_violations": violations, "violation_examples": examples[:6]}


async def soak(lc, args) -> dict:
    for i in range(2):
        _tenant(lc, args, f"s{i}")
    att, det = [], []
    width = min(4, len(lc.nodes["node-0"].node.gpus))   # 1..4 GPUs per attach (fewer if small)
    for k in range(args.cycles):
        t = f"s{k % 2}"
        n = (k % width) + 1
        t0 = time.perf_counter()
        code, b = await lc.add("default", t, n, entire=k % 3 == 0)
        t1 = time.perf_counter()
        if code != 200:
            raise RuntimeError(f"cycle {k}: {code} {b}")
        code, _ = await lc.remove("default", t, [d["uuid"] for d in b["devices"]])
        if code != 200:
            raise RuntimeError(f"cycle {k} detach: {code}")
        att.append((t1 - t0) * 1e3)
        det.append((time.perf_counter() - t1) * 1e3)
    node = lc.nodes["node-0"].node
    if getattr(args, "sandbox", None) is not None:
        # real node: what is left in each tenant's own /dev, seen through its mount namespace
        orphan_nodes = sum(len(_real_dev_nodes(pid)) for pid in args.tenant_pids.values())
    else:
        orphan_nodes = sum(len(node.container_devices(c)) for t in ("s0", "s1")
                           for c in lc.container_ids("default", t))
    orphan_rules = 0
    for t in ("s0", "s1"):
        orphan_rules += len(await lc.audit("default", t))
    return {"cycles": args.cycles, "attach_p50_ms": round(pct(att, 0.5), 3),
            "attach_p99_ms": round(pct(att, 0.99), 3), "detach_p50_ms": round(pct(det, 0.5), 3),
            "detach_p99_ms": round(pct(det, 0.99), 3), "orphaned_cgroup_entries": orphan_rules,
            "orphaned_device_nodes": orphan_nodes,
            "placeholders_left": len(lc.cluster.placeholders()),
            "gpus_still_allocated": len(node.allocated)}


def contention_processes(args) -> dict:
    """The contention scenario against the deployment shape: master, worker and control plane
    as separate processes (ProcessCluster, deployed as shipped: mTLS + authz), one client thread
    per Pod issuing its adds/removes over HTTP concurrently with the others. Invariants after
    every round, read through the public APIs only: each Pod's hot-mounted set equals what its
    client attached, no GPU is hot-mounted twice, the placeholders hold exactly the hot-mounted
    GPUs, and every Pod's audit is clean."""
    from concurrent.futures import ThreadPoolExecutor

    from gpumounter_amd.fakes.deployment import ProcessCluster
    tenants = [f"c{i}" for i in range(4)]
    lat, ok, fail, problems = [], 0, 0, []
    mine = {t: [] for t in tenants}          # client-side record: [(uuids, entire)]
    rnds = {t: random.Random(args.seed * 31 + i) for i, t in enumerate(tenants)}
    with ProcessCluster(amdsmi_lib=args.amdsmi, cgroup_mode=args.cgroup) as pc:
        for t in tenants:
            pc.tenant(t)

        def op(t):
            rnd = rnds[t]
            if mine[t] and rnd.random() < 0.5:
                groups = mine[t]
                if any(e for _, e in groups):
                    pick = list(groups)
                else:
                    pick = rnd.sample(groups, rnd.randint(1, len(groups)))
                code, _ = pc.remove("default", t, [u for g, _ in pick for u in g], force=True)
                if code == 200:
                    for g in pick:
                        groups.remove(g)
                return code, None
            n, entire = rnd.randint(1, 4), rnd.random() < 0.3
            t0 = time.perf_counter()
            code, b = pc.add("default", t, n, entire=entire)
            ms = (time.perf_counter() - t0) * 1e3
            if code == 200:
                uu = [d["uuid"] for d in b["devices"]]
                mine[t].extend([(uu, True)] if entire else [([u], False) for u in uu])
            return code, ms

        t_start = time.perf_counter()
        with ThreadPoolExecutor(len(tenants)) as ex:
            for _ in range(args.rounds):
                for code, ms in ex.map(op, tenants):
                    ok += code == 200
                    fail += code != 200
                    if code == 200 and ms is not None:
                        lat.append(ms)
                hot_all = []
                for t in tenants:
                    code, g = pc.pod_gpus("default", t)
                    hot = sorted(x["uuid"] for x in g.get("gpus", [])
                                 if x.get("source") == "hot-mount")
                    hot_all += hot
                    want = sorted(u for grp, _ in mine[t] for u in grp)
                    if hot != want:
                        problems.append(f"{t}: ledger {hot} != attached {want}")
                    issues = pc.audit("default", t)
                    if issues:
                        problems.append(f"{t}: audit {issues}")
                if len(hot_all) != len(set(hot_all)):
                    problems.append(f"GPU hot-mounted twice: {sorted(hot_all)}")
                held = sum(int(c.get("resources", {}).get("limits", {}).get("amd.com/gpu", 0))
                           for p in pc.placeholders() for c in p["spec"]["containers"])
                if held != len(hot_all):
                    problems.append(f"placeholders hold {held} GPUs, {len(hot_all)} hot-mounted")
        elapsed = time.perf_counter() - t_start
    return {"rounds": args.rounds, "ops_ok": ok, "ops_refused": fail,
            "ops_per_s": round((ok + fail) / elapsed, 1),
            "attach_p50_ms": round(pct(lat, 0.5), 3) if lat else None,
            "attach_p99_ms": round(pct(lat, 0.99), 3) if lat else None,
            "invariant_violations": len(problems), "violation_examples": problems[:5]}


def _gpus_held(p: dict) -> int:
    """GPUs a bound placeholder holds: its amd.com/gpu limit, or (DRA) its claim's device count
    (the gpumounter.amd.com/gpus annotation the claim was built from)."""
    if not p["spec"].get("nodeName"):
        return 0
    lim = sum(int(c.get("resources", {}).get("limits", {}).get("amd.com/gpu", 0))
              for c in p["spec"]["containers"])
    if lim or not p["spec"].get("resourceClaims"):
        return lim
    return int((p["metadata"].get("annotations") or {}).get("gpumounter.amd.com/gpus", "0"))


CHAOS_FAULTS = ("ledger_reserve:0.04,placeholder_wait:0.03,cgroup_rule:0.04,devnodes:0.04,"
                "cgroup_rule:0.04:after,busy_check:0.03,unmount:0.04,ledger_release:0.04,"
                "ledger_release:0.04:after")


def _http_json(method: str, url: str, body=None):
    """One JSON request to the hermetic apiserver: (status, decoded body or {})."""
    from gpumounter_amd.fakes.deployment import _http
    code, raw = _http(method, url, json.dumps(body).encode() if body is not None else None,
                      {"Content-Type": "application/json"} if body is not None else None)
    try:
        return code, json.loads(raw) if raw else {}
    except ValueError:
        return code, {}


def chaos(args) -> dict:
    """Contention under failure, against the deployment shape (ProcessCluster, mTLS + authz):
    four Pods attach and detach concurrently over HTTP while the worker injects faults at every
    mutating stage (GM_FAULT, before and after each side effect) and is SIGKILLed with requests
    in flight every ``--kill-every`` rounds, then restarted. After every round, once the node
    has converged, the invariants are read through the public APIs only:
    * every Pod's audit is clean: the device rules and nodes in its containers are exactly its
      ledger's hot-mounted GPUs (nothing leaked into a container, nothing missing);
    * no GPU is hot-mounted twice, and the placeholders hold exactly the hot-mounted GPUs;
    * a Pod whose requests all succeeded since the last check holds exactly what its client
      attached and did not remove (a failed request may or may not have taken effect, so after
      one the client re-reads its state from the ledger).
    ``converge_ms`` is how long the node took to satisfy the first two after a round.

    ``--busy``: every hot-mounted GPU is in use by a process of its tenant that ignores SIGTERM
    (listed in the mock amdsmi's process table, a real child process in the container's
    cgroup.procs), so every removal is a force removal that has to kill it. Two more
    invariants: a removal answered with success named only processes that are gone, and a GPU
    is never released while the process that used it still runs (reference order: kill, then
    delete the slave pods and wait for them, pkg/util/util.go:112-143,
    pkg/util/gpu/allocator/allocator.go:128-156)."""
    from concurrent.futures import ThreadPoolExecutor

    from gpumounter_amd.fakes.deployment import ProcessCluster
    tenants = [f"x{i}" for i in range(4)]
    rnds = {t: random.Random(args.seed * 17 + i) for i, t in enumerate(tenants)}
    mine = {t: [] for t in tenants}
    leases = {t: {} for t in tenants}        # uuid -> (earliest, latest) expiry of its lease
    leased, expired = [0], [0]
    certain = {t: True for t in tenants}
    resyncs = {t: 0 for t in tenants}   # ledger reads left before a failed tenant is certain
    answered = {t: [] for t in tenants}      # (code, [(placeholder, uuid tail)], lease) per attach
    ok = failed = kills = restarts = master_kills = recreates = kubelet_restarts = 0
    recreated: set = set()
    problems, converge = [], []
    api_faults = [0]
    codes: Dict[int, int] = {}
    env = {"GM_FAULT": CHAOS_FAULTS, "GM_RECONCILE_PERIOD_S": str(args.reconcile_period),
           "GM_WARM_POOL_SIZE": str(args.warm_pool), "GM_PLACEMENT_ENFORCE": args.placement}
    if args.pool_priority_class:
        env["GM_POOL_PRIORITY_CLASS"] = args.pool_priority_class
    if args.placeholder_binding:
        env["GM_PLACEHOLDER_BINDING"] = args.placeholder_binding
    if args.no_placeholder_priority:
        env["GM_PLACEHOLDER_PRIORITY_CLASS"] = ""       # the reference's priority 0
    if args.log_dir:
        env["GM_LOG_LEVEL"] = "DEBUG"      # kept logs are for post-mortems
    busy = _BusyTenants(tenants, args.busy_pool) if args.busy else None
    if busy is not None:
        env.update({"GM_AMDSMI_MOCK_PROCS": busy.table, "GM_BUSY_DETECTION": "both",
                    "GM_KILL_GRACE_S": str(args.kill_grace)})
    with ProcessCluster(amdsmi_lib=args.amdsmi, cgroup_mode=args.cgroup, worker_env=env,
                        master_env={"GM_LOG_LEVEL": "DEBUG"} if args.log_dir else None,
                        gpu_api=args.gpu_api, log_dir=args.log_dir,
                        latency=args.latency, lazy_checkpoint=args.lazy_checkpoint) as pc, \
            (busy or contextlib.nullcontext()):
        for t in tenants:
            pc.tenant(t, pids={"main": busy.pids(t)} if busy else None)
        if args.api_fault_rate:
            pc.api_faults(args.api_fault_rate, args.seed)
        api = pc.info["api_url"]
        preemptors: List[str] = []
        preempted = [0, 0]          # preemptors created, of them bound
        if args.preempt_rate:
            code, _ = _http_json("POST", f"{api}/apis/scheduling.k8s.io/v1/priorityclasses",
                                 {"metadata": {"name": "chaos-high"}, "value": 1000})
            if code not in (201, 409):
                raise RuntimeError(f"priority class create: {code}")

        def preemptor_churn(rnd_i):
            """Delete last round's preemptor; maybe send a new one (see --preempt-rate)."""
            while preemptors:
                name = preemptors.pop()
                code, body = _http_json("GET", f"{api}/api/v1/namespaces/default/pods/{name}")
                if code == 200 and body.get("spec", {}).get("nodeName"):
                    preempted[1] += 1
                for _ in range(20):      # the apiserver's injected faults hit these too
                    code, _ = _http_json("DELETE", f"{api}/api/v1/namespaces/default/pods/{name}",
                                         {"gracePeriodSeconds": 0})
                    if code in (200, 404):
                        break
            rnd = random.Random(args.seed * 131 + rnd_i)
            if rnd.random() < args.preempt_rate:
                name = f"preemptor-{rnd_i}"
                want = args.preempt_gpus or rnd.randint(1, 2)
                code, _ = _http_json("POST", f"{api}/api/v1/namespaces/default/pods", {
                    "metadata": {"name": name},
                    "spec": {"priorityClassName": "chaos-high",
                             "nodeSelector": {"kubernetes.io/hostname": "node-0"},
                             "containers": [{"name": "c", "image": "x:1", "resources": {
                                 "limits": {"amd.com/gpu": str(want)}}}]}})
                preemptors.append(name)     # a failed POST may have taken effect: delete it too
                if code == 201:
                    preempted[0] += 1

        def op(t):
            rnd = rnds[t]
            try:
                # leased GPUs are left to their lease: the check sees whether it ended
                groups = [g for g in mine[t] if not set(g[0]) & set(leases[t])]
                if groups and rnd.random() < 0.5:
                    pick = list(groups) if any(e for _, e in groups) else \
                        rnd.sample(groups, rnd.randint(1, len(groups)))
                    code, b = pc.remove("default", t, [u for g, _ in pick for u in g], force=True)
                    if code == 200:
                        for g in pick:
                            mine[t].remove(g)
                        if busy is not None:
                            busy.check_killed(t, b.get("killed_pids") or [], problems)
                    return t, code
                n, entire = rnd.randint(1, 3), rnd.random() < 0.3
                lease = round(rnd.uniform(0.1, 0.5), 2) if rnd.random() < args.lease_rate else 0
                sent = time.monotonic()
                code, b = pc.add("default", t, n, entire=entire, lease_s=lease)
                answered[t].append((code, [(d.get("placeholder"), d["uuid"][-4:])
                                           for d in (b.get("devices") or [])]
                                    if isinstance(b, dict) else None, lease))
                if code == 200:
                    uu = [d["uuid"] for d in b["devices"]]
                    # a GPU attached again was in an earlier lease of this tenant: that lease
                    # has ended (the ledger never holds a GPU twice)
                    ended = set(uu) & set(leases[t])
                    if ended:
                        mine[t] = [g for g in mine[t] if not set(g[0]) & ended]
                        for u in ended:
                            leases[t].pop(u)
                        expired[0] += len(ended)
                    mine[t].extend([(uu, True)] if entire else [([u], False) for u in uu])
                    if lease:   # the worker's lease clock started between sending and answer
                        # (by placeholder: a GPU re-attached by a later attach whose answer was
                        # lost is held by another placeholder, not by the lease)
                        leases[t].update({d["uuid"]: (sent + lease, time.monotonic() + lease,
                                                      d.get("placeholder"))
                                          for d in b["devices"]})
                        leased[0] += 1
                return t, code
            except Exception:  # noqa: BLE001 - the master's connection dropped mid-kill
                return t, -1

        holders = {}    # tenant → {uuid: placeholder holding it} as of the last ledger()
        lease_now = {}  # tenant → {uuid: lease_expires on the ledger} as of the last ledger()

        def still_leased(t, u) -> bool:
            """The ledger still shows GPU ``u`` under the lease the client recorded (not a
            later, unleased claim of the same warm-pool placeholder whose answer was lost)."""
            exp = lease_now.get(t, {}).get(u)
            if not exp:
                return False
            at = time.monotonic() + (exp - time.time())
            return leases[t][u][0] - 1.0 <= at <= leases[t][u][1] + 1.0

        ledger_err = {}     # tenant → (code, answer, seconds) of its last failed ledger read

        def ledger(t):
            t0 = time.perf_counter()
            try:
                code, g = pc.pod_gpus("default", t)
            except Exception as e:  # noqa: BLE001 - the master restarting, a read timeout
                code, g = -1, {"error": repr(e)}
            if code != 200:
                ledger_err[t] = (code, str(g)[:200], round(time.perf_counter() - t0, 3))
                return None
            hm = [x for x in g.get("gpus", []) if x.get("source") == "hot-mount"]
            holders[t] = {x["uuid"]: x.get("pod_name") for x in hm}
            lease_now[t] = {x["uuid"]: x.get("lease_expires") for x in hm}
            return sorted(x["uuid"] for x in hm)

        why = [""]

        def converged():
            hot_all = []
            for t in tenants:
                hot = ledger(t)
                if hot is None:
                    why[0] = f"{t}: no ledger view {ledger_err.get(t)}"
                    return False
                issues = pc.audit("default", t)
                if issues:
                    why[0] = f"{t}: audit {issues[:3]}"
                    return False
                hot_all += hot
            # every placeholder left must be bound and hold GPUs of the hot-mounted set: an
            # unbound one (its attach died) would be admitted later and hand a Pod GPUs nobody
            # asked for
            phs = [p for p in pc.placeholders()
                   if (p["metadata"].get("annotations") or {}).get(
                       "gpumounter.amd.com/mount-mode") != "standby"]     # warm pool
            unbound = [p["metadata"]["name"] for p in phs if not p["spec"].get("nodeName")]
            if unbound:
                why[0] = f"unbound placeholders left: {unbound}"
                return False
            held = sum(_gpus_held(p) for p in phs)
            if len(hot_all) != len(set(hot_all)) or held != len(hot_all):
                why[0] = (f"hot {sorted(hot_all)} vs placeholders holding {held}: "
                          f"{[(p['metadata']['name'], (p['metadata'].get('annotations') or {}).get('gpumounter.amd.com/mount-mode'), p['status'].get('phase')) for p in phs]}")
                return False
            return True

        def gpu_views():
            out = {}
            for t in tenants:
                code, g = pc.pod_gpus("default", t)
                out[t] = {x["uuid"]: x["index"] for x in g.get("gpus", [])
                          if x.get("source") == "hot-mount"} if code == 200 else None
            return out

        with ThreadPoolExecutor(len(tenants)) as ex:
            for rnd_i in range(args.rounds):
                if busy is not None:
                    busy.publish(gpu_views())
                futs = [ex.submit(op, t) for t in tenants]
                if args.preempt_rate:
                    preemptor_churn(rnd_i)
                if args.recreate_rate and random.Random(rnd_i * 11 + 3).random() < args.recreate_rate:
                    # a tenant Pod is deleted and recreated under its name (new UID) mid-round
                    t = random.Random(rnd_i + 9).choice(tenants)
                    pc.recreate_pod("default", t)
                    recreated.add(t)
                    recreates += 1
                if args.kubelet_restart_every and \
                        rnd_i % args.kubelet_restart_every == args.kubelet_restart_every - 1:
                    pc.restart_kubelet("node-0", down_s=0.05)
                    kubelet_restarts += 1
                if args.restart_rate and random.Random(rnd_i * 7 + 1).random() < args.restart_rate:
                    # a tenant's container crashes and comes back while requests are in flight
                    pc.restart_container("default", random.Random(rnd_i).choice(tenants))
                    restarts += 1
                if args.master_kill_every and \
                        rnd_i % args.master_kill_every == args.master_kill_every - 1:
                    time.sleep(random.Random(rnd_i + 5).uniform(0.0, 0.004))
                    pc.restart_master()             # SIGKILL with requests in flight
                    master_kills += 1
                if args.kill_every and rnd_i % args.kill_every == args.kill_every - 1:
                    time.sleep(random.Random(rnd_i).uniform(0.0, 0.004))
                    pc.kill_worker("node-0")        # SIGKILL with requests in flight
                    kills += 1
                    results = [f.result() for f in futs]
                    pc.restart_worker("node-0")
                else:
                    results = [f.result() for f in futs]
                for t in recreated:
                    certain[t] = False
                    resyncs[t] = 2
                recreated.clear()
                for t, code in results:
                    codes[code] = codes.get(code, 0) + 1
                    ok += code == 200
                    failed += code not in (200, 400, 403)   # 400/403 are answers, not failures
                    if code not in (200, 400, 403):
                        # resynchronised from the ledger at this check and the next: a request
                        # whose master was killed under it goes on in the worker (its operations
                        # are shielded) and can finish after this round's read of the ledger
                        certain[t] = False
                        resyncs[t] = 2
                if args.api_fault_rate:
                    api_faults[0] += pc.api_faults(0)        # the checks read a healthy API
                t0 = time.perf_counter()
                while not converged():
                    if time.perf_counter() - t0 > 20:
                        problems.append(f"round {rnd_i}: not converged after 20 s: {why[0]}")
                        if args.log_dir:      # what the worker is waiting for, and the state
                            with open(os.path.join(args.log_dir,
                                                   f"tasks_round{rnd_i}.txt"), "w") as fh:
                                fh.write(pc.worker_tasks())
                            with open(os.path.join(args.log_dir,
                                                   f"state_round{rnd_i}.json"), "w") as fh:
                                json.dump({"audit": {t: pc.audit("default", t) for t in tenants},
                                           "pod_gpus": {t: pc.pod_gpus("default", t)
                                                        for t in tenants},
                                           "placeholders": [
                                               {"name": p["metadata"]["name"],
                                                "rv": p["metadata"].get("resourceVersion"),
                                                "annotations": p["metadata"].get("annotations"),
                                                "phase": p["status"].get("phase")}
                                               for p in pc.placeholders()]}, fh, indent=1)
                        break
                    time.sleep(0.05)
                converge.append((time.perf_counter() - t0) * 1e3)
                if busy is not None:
                    busy.check_booked(rnd_i, gpu_views(), problems)
                for t in tenants:
                    hot = ledger(t) or []
                    now = time.monotonic()
                    # a lease past its expiry is gone, one within it is still there; one that
                    # expires around now may be either (it is settled at the next check)
                    overdue = [u for u, (_, hi, _) in leases[t].items()
                               if now - hi > args.lease_slack]
                    # after a lost answer (not certain) the tenant may have re-attached the GPU
                    # under the same placeholder without a lease: only the ledger's own lease
                    # annotation tells (the client resyncs from the ledger further down)
                    late = sorted(u for u in overdue if u in hot and
                                  holders.get(t, {}).get(u) == leases[t][u][2] and
                                  (certain[t] or still_leased(t, u)))
                    if late:
                        problems.append(f"round {rnd_i} {t}: leases expired more than "
                                        f"{args.lease_slack} s ago still attached: {late}; "
                                        f"held by {[holders.get(t, {}).get(u) for u in late]}; "
                                        f"last answers {answered[t][-4:]}")
                    gone = set(overdue) - set(late)
                    for u in gone:
                        leases[t].pop(u)
                        expired[0] += 1
                    if gone:
                        mine[t] = [g for g in mine[t] if not set(g[0]) & gone]
                    fuzzy = {u for u, (lo, _, _) in leases[t].items() if lo <= now}
                    hot = [u for u in hot if u not in fuzzy]
                    want = sorted(u for grp, _ in mine[t] for u in grp if u not in fuzzy)
                    if certain[t] and hot != want:
                        mine_phs = [(p["metadata"]["name"],
                                     {k.split("/")[-1]: v for k, v in
                                      (p["metadata"].get("annotations") or {}).items()
                                      if k.split("/")[-1] in ("attach-id", "mount-mode",
                                                              "worker-incarnation")})
                                    for p in pc.placeholders()
                                    if (p["metadata"].get("annotations") or {}).get(
                                        "gpumounter.amd.com/owner-name") == t]
                        problems.append(f"round {rnd_i} {t}: ledger {hot} != attached {want}; "
                                        f"placeholders {mine_phs}; answered {answered[t]}")
                    if not certain[t]:
                        # resynchronise the client from the ledger: single mounts per GPU (an
                        # entire mount's GPUs are removed together; the ledger's mount type says)
                        code, g = pc.pod_gpus("default", t)
                        mine[t] = [([x["uuid"]], False) for x in g.get("gpus", [])
                                   if x.get("source") == "hot-mount"]
                        ph = {x.get("pod_name") for x in g.get("gpus", [])
                              if x.get("source") == "hot-mount"}
                        if len(ph) < len(mine[t]):      # fewer placeholders than GPUs: entire
                            mine[t] = [([u for grp, _ in mine[t] for u in grp], True)]
                        held_now = {x["uuid"]: x.get("pod_name") for x in g.get("gpus", [])
                                    if x.get("source") == "hot-mount"}
                        # a lease still stands if its placeholder holds the GPU *with that lease*:
                        # a warm-pool placeholder given back and claimed again (by this Pod's
                        # later attach, answer lost) has the same name and no lease
                        on_ledger = {x["uuid"]: x.get("lease_expires")
                                     for x in g.get("gpus", []) if x.get("source") == "hot-mount"}

                        def same_lease(u, e):
                            exp = on_ledger.get(u)
                            if not exp:
                                return False
                            at = time.monotonic() + (exp - time.time())
                            return e[0] - 1.0 <= at <= e[1] + 1.0
                        leases[t] = {u: e for u, e in leases[t].items()
                                     if held_now.get(u) == e[2] and same_lease(u, e)}
                        # a leased attach whose answer was lost: its lease is on the ledger
                        for x in g.get("gpus", []):
                            exp = x.get("lease_expires")
                            if x.get("source") == "hot-mount" and exp and \
                                    x["uuid"] not in leases[t]:
                                at = time.monotonic() + (exp - time.time())
                                leases[t][x["uuid"]] = (at, at, x.get("pod_name"))
                        resyncs[t] = resyncs.get(t, 1) - 1
                        certain[t] = resyncs[t] <= 0
                if args.api_fault_rate:
                    pc.api_faults(args.api_fault_rate, args.seed * 1000 + rnd_i)
        metrics = pc.worker_metrics()
        busy_report = busy.report() if busy is not None else {}
        code, preempt = _http_json("GET", f"{api}/_fake/preemptions")
        if code != 200:
            raise RuntimeError(f"preemptions: {code}")
        if preempt["victims"]["placeholder"]:
            # the shipped floor class outranks every preemptor here: a placeholder that books
            # a tenant's GPU is never a victim (only standbys at the low class may be)
            problems.append(f"{preempt['victims']['placeholder']} placeholder(s) booking a "
                            f"tenant's GPU preempted")
    injected = sum(float(ln.split()[-1]) for ln in metrics.splitlines()
                   if ln.startswith("gm_requests_total{") and 'result="INTERNAL"' in ln)
    return {"rounds": args.rounds, "worker_kills": kills, "master_kills": master_kills,
            "container_restarts": restarts, "pod_recreates": recreates,
            "kubelet_restarts": kubelet_restarts,
            "ops_ok": ok,
            "ops_failed": failed, "internal_errors_since_last_restart": injected,
            "converge_p50_ms": round(pct(converge, 0.5), 1),
            "converge_max_ms": round(max(converge), 1),
            "invariant_violations": len(problems), "violation_examples": problems[:5],
            "preemptors": preempted[0], "preemptors_bound": preempted[1],
            "preempted": preempt["victims"],
            "faults": CHAOS_FAULTS, "api_fault_rate": args.api_fault_rate,
            "reconcile_period_s": args.reconcile_period, "placement": args.placement,
            "api_faults_served": api_faults[0],
            "answers": {str(k): v for k, v in sorted(codes.items())},
            "leases": {"rate": args.lease_rate, "attached": leased[0], "seen_expired": expired[0],
                       "slack_s": args.lease_slack},
            **busy_report}


class _BusyTenants:
    """chaos --busy: per tenant, a pool of processes that ignore SIGTERM (all in the tenant
    container's cgroup.procs from the start); the current one is listed in the mock amdsmi
    process table as the user of every GPU the tenant holds."""

    def __init__(self, tenants: List[str], pool: int):
        import tempfile
        self.dir = tempfile.mkdtemp(prefix="gm-busy-")
        self.table = os.path.join(self.dir, "procs")
        open(self.table, "w").close()
        self.procs = {t: [subprocess.Popen(["sh", "-c", "trap '' TERM; exec sleep 3600"],
                                           stdin=subprocess.DEVNULL,
                                           start_new_session=True) for _ in range(pool)]
                      for t in tenants}
        self.cur = {t: 0 for t in tenants}
        self.listed: Dict[int, tuple] = {}       # GPU index -> (tenant, Popen) as published
        self.kills_seen = 0
        self.exhausted = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc) -> None:
        for ps in self.procs.values():
            for p in ps:
                if p.poll() is None:
                    p.kill()
                    p.wait()
        shutil.rmtree(self.dir, ignore_errors=True)

    def pids(self, t: str) -> List[int]:
        return [p.pid for p in self.procs[t]]

    def _current(self, t: str):
        ps = self.procs[t]
        while self.cur[t] < len(ps) and ps[self.cur[t]].poll() is not None:
            self.cur[t] += 1                     # killed by a force removal: the next one
        if self.cur[t] >= len(ps):
            self.exhausted += 1
            return None
        return ps[self.cur[t]]

    def publish(self, views: Dict[str, Optional[dict]]) -> None:
        """Every GPU a tenant holds is in use by its current process."""
        self.listed = {}
        lines = []
        for t, v in views.items():
            p = self._current(t)
            if p is None or not v:
                continue
            for idx in sorted(v.values()):
                self.listed[idx] = (t, p)
                lines.append(f"{idx} {p.pid} 4096 sleep\n")
        tmp = self.table + ".tmp"
        with open(tmp, "w") as fh:
            fh.write("".join(lines))
        os.replace(tmp, self.table)

    def check_killed(self, t: str, pids: List[int], problems: list) -> None:
        """A removal answered with success: the processes it killed are gone."""
        by_pid = {p.pid: p for p in self.procs[t]}
        for pid in pids:
            self.kills_seen += 1
            p = by_pid.get(pid)
            if p is None:
                problems.append(f"{t}: removal killed {pid}, not one of the tenant's processes")
            elif p.poll() is None:
                time.sleep(0.05)                 # reaped by us, not by the worker: allow a beat
                if p.poll() is None:
                    problems.append(f"{t}: removal answered success while killed PID {pid} "
                                    f"still runs")

    def check_booked(self, rnd_i: int, views: Dict[str, Optional[dict]], problems: list) -> None:
        """A GPU whose listed process still runs is still its tenant's (never released)."""
        for idx, (t, p) in self.listed.items():
            if p.poll() is None and views.get(t) is not None and idx not in views[t].values():
                problems.append(f"round {rnd_i}: GPU {idx} released from {t} while its process "
                                f"{p.pid} still runs")

    def report(self) -> dict:
        return {"busy": {"force_kills_answered": self.kills_seen,
                         "processes_killed": sum(p.poll() is not None
                                                 for ps in self.procs.values() for p in ps),
                         "pool_exhausted_rounds": self.exhausted}}


async def placement(lc, args) -> dict:
    """Placement quality on a fragmented node, as a device plugin that ignores gpumounter's
    hint leaves it. Four background pods grow and shrink by single GPUs at random; between
    their moves a probe pod attaches N ∈ {1, 2, 4} GPUs (entire or single mount, at random) and
    detaches again. Each attach is compared with the best set the free GPUs allowed at that
    moment (hive split ≫ non-xGMI pair ≫ NUMA split, hw/topology.py)."""
    rnd = random.Random(args.seed)
    bg = [f"bg{i}" for i in range(4)]
    for t in bg + ["probe"]:
        _tenant(lc, args, t)
    node = lc.nodes["node-0"].node
    svc = lc.nodes["node-0"].worker.service
    links = lc.inventory.links()
    table = {g.index: g for g in node.gpus}
    by_bdf = {g.bdf: g for g in node.gpus}
    stats = {n: {"attaches": 0, "optimal": 0, "numa_possible": 0, "numa_packed": 0,
                 "one_hive": 0, "ms": []} for n in (1, 2, 4)}
    for _ in range(args.rounds):
        for t in bg:
            st = await svc.pod_state(lc.cluster.get("default", t))
            if st.hot and (rnd.random() < 0.45 or len(node.allocated) >= len(node.gpus) - 2):
                await lc.remove("default", t, [rnd.choice(st.hot).uuid], force=True)
            elif len(node.allocated) < len(node.gpus) - 2:
                await lc.add("default", t, 1)
        for n in (1, 2, 4):
            free = [g for g in node.gpus if node.device_id(g) not in node.allocated]
            best = topology.choose(free, n, links)
            if best is None:
                continue
            t0 = time.perf_counter()
            code, b = await lc.add("default", "probe", n, entire=rnd.random() < 0.5)
            ms = (time.perf_counter() - t0) * 1e3
            if code != 200:
                continue          # a background move took a GPU meanwhile: not a placement
            got = [by_bdf[d["bdf"]].index for d in b["devices"]]
            score, hives, numa, _ = topology.score_set(table, links, got)
            s = stats[n]
            s["attaches"] += 1
            s["ms"].append(ms)
            s["optimal"] += score <= best.score + 1e-6
            s["one_hive"] += hives == 1
            if best.numa_nodes == 1:
                s["numa_possible"] += 1
                s["numa_packed"] += numa == 1
            code, _ = await lc.remove("default", "probe", [d["uuid"] for d in b["devices"]])
            if code != 200:
                raise RuntimeError(f"probe detach: {code}")
    out = {}
    for n, s in stats.items():
        ms = s.pop("ms")
        out[str(n)] = dict(s, attach_p50_ms=round(pct(ms, 0.5), 3) if ms else None,
                           attach_p99_ms=round(pct(ms, 0.99), 3) if ms else None)
    m = svc.metrics
    return {"per_n": out, "placement_corrections": int(m.placement_corrections._value.get()),
            "placement_mismatch": int(m.placement_mismatch._value.get()),
            "audit_issues": sum([len(await lc.audit("default", t)) for t in bg + ["probe"]])}


SCENARIOS = {"scale": scale, "contention": contention, "soak": soak, "placement": placement,
             "chaos": None}     # process deployment only (see chaos())


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("scenario", choices=sorted(SCENARIOS))
    ap.add_argument("--amdsmi", default="mock", help='"mock" (default) or "" for libamd_smi')
    ap.add_argument("--cgroup", choices=("v1", "v2"), default="v2")
    ap.add_argument("--latency", choices=("zero", "realistic", "teardown"), default="zero",
                    help="control-plane latency model; teardown: zero, but the kubelet frees "
                         "a deleted Pod's devices 50 ms after the DELETE (chaos only)")
    ap.add_argument("--placement", choices=("auto", "hint", "trim"), default="auto")
    ap.add_argument("--alloc-policy", choices=("first-free", "random", "topology"),
                    default="first-free",
                    help="the fake node's device choice: first free in device order; random "
                         "(the kubelet's pick without GetPreferredAllocation); or a plugin's own "
                         "pod-blind topology choice")
    ap.add_argument("--device-plugin", action="store_true")
    ap.add_argument("--warm-pool", type=int, default=0)
    ap.add_argument("--lazy-checkpoint", action="store_true",
                    help="chaos: the fake kubelet keeps a deleted Pod in its device-manager "
                         "checkpoint until the next Allocate, as a real one does")
    ap.add_argument("--placeholder-binding", default="", choices=("", "scheduler", "direct"),
                    help="chaos: GM_PLACEHOLDER_BINDING for the workers (default: the shipped)")
    ap.add_argument("--no-placeholder-priority", action="store_true",
                    help="chaos: placeholders without the floor PriorityClass (the reference's "
                         "priority 0), the negative control for --preempt-rate")
    ap.add_argument("--preempt-gpus", type=int, default=0,
                    help="chaos: GPUs each --preempt-rate Pod requests (0: 1 or 2 at random)")
    ap.add_argument("--preempt-rate", type=float, default=0.0,
                    help="chaos: per round, the chance that a Pod of priority 1000 (above every "
                         "tenant, below the placeholders' floor) asks for 1-2 GPUs on the node; "
                         "it is deleted the next round. It may take free GPUs or preempt idle "
                         "low-class standbys, never a placeholder that books a tenant's GPU "
                         "(checked through the fake scheduler's victims)")
    ap.add_argument("--pool-priority-class", default="",
                    help="GM_POOL_PRIORITY_CLASS for the workers (chaos, processes): e.g. "
                         "gpumounter-standby, idle standbys preemptible and yielded to attaches")
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--cycles", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gpu-api", choices=("device-plugin", "dra"), default="device-plugin",
                    help="chaos: GPUs from the device plugin or from a DRA driver")
    ap.add_argument("--api-fault-rate", type=float, default=0.0,
                    help="chaos: Pod/ResourceClaim requests to the apiserver fail at random at "
                         "this rate (500/503/429, half after taking effect)")
    ap.add_argument("--restart-rate", type=float, default=0.0,
                    help="chaos: per round, the probability that a tenant's container restarts "
                         "with requests in flight")
    ap.add_argument("--master-kill-every", type=int, default=0,
                    help="chaos: SIGKILL and restart the master with requests in flight every N "
                         "rounds")
    ap.add_argument("--recreate-rate", type=float, default=0.0,
                    help="chaos: per round, the probability that a tenant Pod is deleted and "
                         "recreated under the same name with requests in flight")
    ap.add_argument("--kubelet-restart-every", type=int, default=0,
                    help="chaos: restart the kubelet (PodResources socket recreated) every N "
                         "rounds")
    ap.add_argument("--reconcile-period", type=float, default=0.5,
                    help="chaos: the worker's periodic sweep (GM_RECONCILE_PERIOD_S; shipped 30)")
    ap.add_argument("--faults", action="store_true",
                    help="in-process scenarios: the chaos scenario's stage faults (GM_FAULT) in "
                         "the worker; with --node-ops real every failure path runs against real "
                         "BPF programs and device nodes")
    ap.add_argument("--lease-rate", type=float, default=0.0,
                    help="chaos: the share of attaches made with a 0.1-0.5 s lease (?lease=); a "
                         "lease must have ended within --lease-slack of its expiry")
    ap.add_argument("--lease-slack", type=float, default=1.5,
                    help="chaos --lease-rate: how late an expired lease may still be attached")
    ap.add_argument("--busy", action="store_true",
                    help="chaos: every hot-mounted GPU is in use by a SIGTERM-ignoring process "
                         "of its tenant; removals must kill it before releasing the GPU")
    ap.add_argument("--busy-pool", type=int, default=80,
                    help="chaos --busy: processes per tenant (one is killed per busy removal)")
    ap.add_argument("--kill-grace", type=float, default=0.2,
                    help="chaos --busy: the worker's SIGTERM -> SIGKILL grace (GM_KILL_GRACE_S)")
    ap.add_argument("--log-dir", default="",
                    help="chaos: keep the daemons' logs here (default: the cluster's temp dir)")
    ap.add_argument("--kill-every", type=int, default=10,
                    help="chaos: SIGKILL the worker with requests in flight every N rounds")
    ap.add_argument("--node-ops", choices=("emulated", "real"), default="emulated",
                    help="real (root, cgroup2): tenants are processes in their own mount "
                         "namespaces inside real cgroups with a runc-style device program; "
                         "attaches load/update real BPF programs and mknod real nodes")
    ap.add_argument("--deploy", choices=("inprocess", "processes"), default="inprocess",
                    help="processes: daemons as separate processes, clients over HTTP "
                         "(contention only)")
    args = ap.parse_args()
    log.setup("WARNING", json_format=False)
    if args.scenario == "chaos":
        if args.busy and args.lease_rate:
            ap.error("--busy keeps leased GPUs attached (busy leases are kept): no --lease-rate")
        if args.busy and args.recreate_rate:
            ap.error("--busy keeps each tenant's processes in its Pod: no --recreate-rate")
        res = chaos(args)
        res["config"] = {"scenario": "chaos", "deploy": "processes",
                         "amdsmi": args.amdsmi or "libamd_smi", "cgroup": args.cgroup,
                         "warm_pool": args.warm_pool, "gpu_allocation": args.gpu_api,
                         "latency": "zero",
                         "security": "HTTPS + mTLS + TokenReview/SAR authz"}
        print(json.dumps(res))
        return 0
    if args.deploy == "processes":
        if args.scenario != "contention":
            ap.error("--deploy processes runs the contention and chaos scenarios only")
        res = contention_processes(args)
        res["config"] = {"scenario": "contention", "deploy": "processes",
                         "amdsmi": args.amdsmi or "libamd_smi", "cgroup": args.cgroup,
                         "latency": "zero",
                         "security": "HTTPS + mTLS + TokenReview/SAR authz"}
        print(json.dumps(res))
        return 0

    args.sandbox, args.tenant_pids = None, {}
    kw, wov = {}, {"placement_enforce": args.placement, "warm_pool_size": args.warm_pool}
    if args.faults:
        wov["fault"] = CHAOS_FAULTS
    if args.node_ops == "real":
        from gpumounter_amd.fakes.realnode import RealNodeSandbox
        args.cgroup = "v2"
        args.sandbox = RealNodeSandbox().__enter__()
        kw = {"cgroup_root": args.sandbox.cgroup_root, "devnode_mode": "procroot"}
        wov["bpf_pin_dir"] = args.sandbox.bpffs

    async def run():
        lat = LatencyModel.realistic() if args.latency == "realistic" else \
            LatencyModel(teardown_ms=50.0) if args.latency == "teardown" else LatencyModel()
        async with LocalCluster(amdsmi_lib=args.amdsmi, cgroup_mode=args.cgroup, latency=lat,
                                device_plugin=args.device_plugin, worker_overrides=wov,
                                alloc_policy=args.alloc_policy, **kw) as lc:
            # one process holds the fakes, the worker and the master here: freeze the
            # start-up heap as each daemon does on its own (utils/runtime.py), so a full
            # collection of it is not charged to whichever operation it interrupts
            runtime.tune_gc()
            res = await SCENARIOS[args.scenario](lc, args)
            gpus = lc.nodes["node-0"].node.gpus
            res["config"] = {"scenario": args.scenario, "amdsmi": args.amdsmi or "libamd_smi",
                             "node_gpus": len(gpus),
                             "gfx": sorted({g.gfx_target for g in gpus}),
                             "cgroup": args.cgroup, "latency": args.latency,
                             "placement": args.placement, "device_plugin": args.device_plugin,
                             "alloc_policy": args.alloc_policy,
                             "warm_pool": args.warm_pool, "node_ops": args.node_ops,
                             "faults": CHAOS_FAULTS if args.faults else ""}
            if args.sandbox is not None:
                res["kernel"] = _kernel_state(lc, args)
            return res

    try:
        print(json.dumps(asyncio.run(run())))
    finally:
        if args.sandbox is not None:
            args.sandbox.__exit__(None, None, None)
    return 0


def _kernel_state(lc, args) -> dict:
    """After the scenario, read from the kernel: the device programs attached to each tenant's
    cgroup (our wrapper must be gone wherever no GPU is held, the runtime's program back), the
    grants our wrappers still hold, the GPU nodes left in each tenant's /dev, and the pins left
    on the bpffs."""
    import ctypes as C

    from gpumounter_amd import _native
    from gpumounter_amd.node.cgroup import V2BpfBackend
    lib = _native.host()
    out = {"programs": {}, "grants": {}, "dev_nodes": {}}
    node = lc.nodes["node-0"].node
    for name, pid in args.tenant_pids.items():
        (ctr,) = [c for c in node.containers.values() if c.pod_name == name]
        names = []
        for pid_ in V2BpfBackend.attached_ids(ctr.cgroup_dir):
            buf = C.create_string_buffer(32)
            lib.gm_bpf_prog_name(pid_, buf, 32)
            names.append(buf.value.decode())
        out["programs"][name] = names
        out["grants"][name] = sorted(V2BpfBackend("").allowed(ctr.cgroup_dir))
        out["dev_nodes"][name] = _real_dev_nodes(pid)
    out["pins_left"] = sorted(f for f in os.listdir(args.sandbox.bpffs) if f.startswith("gm_"))
    return out


if __name__ == "__main__":
    sys.exit(main())
