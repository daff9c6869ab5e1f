"""A state-machine model of one node's hot-mount ledger (hypothesis ``RuleBasedStateMachine``).

Round 4 found its robustness bugs by grinding chaos seeds (``bench/configs.py chaos``): random
operations against a deployed cluster, invariants checked once a round. This drives the same
in-process deployment (fake apiserver and kubelet, the real worker and master, real sockets)
with rules hypothesis chooses, shrinks what fails to a minimal sequence, and checks the chaos
invariants after *every* step:

* the node converges: every tenant's device rules and nodes are exactly its ledger's GPUs
  (audit), no GPU is hot-mounted twice, the placeholders hold exactly the hot-mounted GPUs and
  every one of them is bound;
* a tenant whose requests all succeeded holds exactly what its client attached and did not
  remove (GPUs under a lease that is ending count either way);
* a lease that ended more than ``SLACK`` seconds ago no longer holds its GPU.

Rules: attach (single or entire mount, with or without a lease), detach, force-remove, let
time pass (leases end), a container restart, a watch relist (410 Gone), the kubelet's status
churn on every placeholder, a worker restart, an attach or detach with one of those events in
flight (and a container restart that only a relist carries), a lost or failed reply on the
next one or two of POST / PATCH / DELETE / GET, an outage that fails every retry of one write
(a lease then ends within ``SLACK`` of the apiserver answering again), and a Pod that outranks
every tenant arriving for GPUs (the scheduler may preempt idle standbys, never a tenant's
placeholder). Variants: the device-plugin ledger, the warm pool, DRA with a warm pool, trim
placement with a warm pool, a warm pool whose standbys are preemptible (low
``pool_priority_class``), direct binding with a warm pool, and a kubelet that frees a deleted
Pod's devices 50 ms late (direct binding, preemptible standbys).

The reference has no locking and no recovery at all (pkg/server/gpu-mount/server.go:34-179,
SURVEY defect 7). Round-4 bug parents this model fails on: ``bench/model_parents.sh``
(profiles/r5_model_check/).

Size: ``GM_MODEL_EXAMPLES`` (default 4) examples of ``GM_MODEL_STEPS`` (default 10) steps per
variant in the CPU suite; sweeps raise both.
"""
import asyncio
import os
import sys
import time

from hypothesis import HealthCheck, Phase, settings
from hypothesis import strategies as st
from hypothesis.stateful import RuleBasedStateMachine, invariant, rule

from gpumounter_amd.fakes.apiserver import LatencyModel
from gpumounter_amd.fakes.harness import ThreadedCluster
from gpumounter_amd.models import pod as podu

TENANTS = ("x0", "x1", "x2")
LEASE = "gpumounter.amd.com/lease-expires"
MODE = "gpumounter.amd.com/mount-mode"
SLACK = 1.5
CONVERGE_S = 15.0

EXAMPLES = int(os.environ.get("GM_MODEL_EXAMPLES", "4"))
STEPS = int(os.environ.get("GM_MODEL_STEPS", "10"))
# GM_MODEL_REFUSALS=off: do not flag an attach refused for too few GPUs while the model
# counts enough free ones (the refill race found by this model is in every tree before its fix;
# off isolates the other findings on old trees, bench/model_parents.sh)
REFUSALS = os.environ.get("GM_MODEL_REFUSALS", "strict") != "off"
# GM_MODEL_SHRINK=0: report the first failing sequence as found (a cluster run is
# nondeterministic: shrinking replays it many times and can end in a Flaky report)
PHASES = [Phase.explicit, Phase.reuse, Phase.generate] + \
    ([Phase.shrink] if os.environ.get("GM_MODEL_SHRINK", "1") != "0" else [])


def check(ok: bool, msg: str) -> None:
    """assert, and print the finding at once: a replay of a nondeterministic run may pass."""
    if not ok:
        print(f"MODEL FINDING: {msg}", file=sys.stderr, flush=True)
        raise AssertionError(msg)


async def _sync(fn, *a, **k):
    """Run a fake-cluster method on the cluster's own loop thread."""
    return fn(*a, **k)


class LedgerModel(RuleBasedStateMachine):
    VARIANT: dict = {}

    def __init__(self) -> None:
        super().__init__()
        # the shipped reconciler period (the harness's default runs none): relists wake it
        self.tc = ThreadedCluster(cgroup_mode="v2", reconcile_period_s=30.0, **self.VARIANT)
        self.lc = self.tc.start()
        for t in TENANTS:
            self.tc.call(_sync(self.lc.tenant, t))
        self.mine = {t: [] for t in TENANTS}          # [(uuids, entire)]
        self.leases = {t: {} for t in TENANTS}        # uuid → (not before, not after, holder)
        self.certain = {t: True for t in TENANTS}
        self.steps = []
        # a Pod class above every tenant's (they have none: priority 0), below the placeholders'
        self.lc.cluster.add_priority_class("model-high", 1000)
        pool = self.VARIANT.get("worker_overrides", {}).get("warm_pool_size", 0)
        if pool:
            self._until(lambda: len(self._worker().pool.standby()) >= pool, 20)

    def teardown(self) -> None:
        self.tc.stop()

    # ------------------------------------------------------------------------ plumbing
    def _worker(self):
        return self.lc.nodes["node-0"].worker

    def _until(self, pred, timeout: float) -> bool:
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            if pred():
                return True
            time.sleep(0.02)
        return pred()

    async def _add(self, t: str, n: int, entire: bool, lease: float):
        q = f"?lease={lease:g}" if lease else ""
        url = (f"{self.lc.master_url}/addgpu/namespace/default/pod/{t}/gpu/{n}/isEntireMount/"
               f"{'true' if entire else 'false'}{q}")
        async with self.lc.session.get(url, headers={"Accept": "application/json"}) as r:
            return r.status, await r.json()

    def _faults(self) -> int:
        return len(getattr(self.lc.cluster, "_faults", ()))

    def _policy_ok(self, t: str, entire: bool):
        """Whether an attach in this mode fits the Pod's current mount mode (one entire mount
        on an unmounted Pod, or singles on a Pod without an entire mount): True, False, or
        None when a failed request or an ending lease leaves it open."""
        if not self.certain[t]:
            return None
        now = time.monotonic()
        sure = [g for g in self.mine[t] if not any(
            self.leases[t].get(u, (now + 1,))[0] <= now + 0.15 for u in g[0])]
        if len(sure) != len(self.mine[t]):
            return None if (not sure if entire else not any(e for _, e in sure)) else False
        return not sure if entire else not any(e for _, e in sure)

    def _answer(self, t: str, code: int, body: dict, excused: bool, n: int = 0,
                entire: bool = False) -> None:
        """A refusal (400, 403, too few GPUs) changes nothing. Any other failure leaves the
        tenant uncertain; without an injected fault or a racing event it is itself a bug."""
        if code in (200, 400, 403):
            return
        if code == 500 and "MountPolicyDenied" in str(body.get("error")):
            check(excused or self._policy_ok(t, entire) is not True,
                  f"{t}: refused as a mount-mode conflict; steps {self.steps}")
            return
        if code == 500 and body.get("add_gpu_result") == "InsufficientGPU":
            check(excused or not REFUSALS or self.room() < n,
                  f"{t}: {n} GPU(s) refused with {self.room()} free; steps {self.steps}")
            return
        check(excused, f"{t}: {code} {body} with no fault injected; steps {self.steps}")
        self.certain[t] = False

    def room(self) -> int:
        """GPUs certainly free: capacity minus every GPU a client may hold (-1: unknown)."""
        if not all(self.certain.values()) or "placement_enforce" in str(self.VARIANT):
            return -1
        cap = len(self.lc.nodes["node-0"].node.gpus)
        used = {u for t in TENANTS for g, _ in self.mine[t] for u in g}
        used |= {u for t in TENANTS for u in self.leases[t]}
        return cap - len(used)

    # ------------------------------------------------------------------------ rules
    @rule(t=st.sampled_from(TENANTS), n=st.integers(1, 3), entire=st.booleans(),
          lease=st.sampled_from([0.0, 0.0, 0.3, 0.8]))
    def attach(self, t, n, entire, lease):
        self._attach(t, n, entire, lease)

    def _attach(self, t, n, entire, lease, event=None, delay=0.0):
        sent = time.monotonic()
        excused = self._faults() > 0 or event is not None
        fits = self._policy_ok(t, entire)
        code, b = self.tc.call(self._racing(self._add(t, n, entire, lease), event, delay))
        self.steps.append(f"attach {t} n={n} entire={entire} lease={lease}"
                          f"{f' racing {event} +{delay * 1e3:g}ms' if event else ''} → {code}")
        self._answer(t, code, b, excused, n, entire)
        if code != 200:
            return
        check(fits is not False, f"{t}: attach (entire={entire}) admitted over a mount-mode "
                                 f"conflict; steps {self.steps}")
        uu = [d["uuid"] for d in b["devices"]]
        ended = set(uu) & set(self.leases[t])     # a GPU back again: its earlier lease ended
        if ended:
            self.mine[t] = [g for g in self.mine[t] if not set(g[0]) & ended]
            for u in ended:
                self.leases[t].pop(u)
        self.mine[t] += [(tuple(uu), True)] if entire else [((u,), False) for u in uu]
        if lease:
            for d in b["devices"]:
                self.leases[t][d["uuid"]] = (sent + lease, time.monotonic() + lease,
                                             d.get("placeholder"))

    # which of the tenant's groups a detach takes: drawn up front as indexes, so the data drawn
    # never depends on what the (nondeterministic) cluster answered before
    PICKS = st.lists(st.integers(0, 7), min_size=1, max_size=3)

    @rule(t=st.sampled_from(TENANTS), force=st.booleans(), picks=PICKS)
    def detach(self, t, force, picks):
        self._detach(t, force, picks)

    def _detach(self, t, force, picks, event=None, delay=0.0):
        # a leased GPU can be detached early, unless its lease may be ending right now
        soon = time.monotonic() + 0.15
        ending = {u for u, (lo, _, _) in self.leases[t].items() if lo <= soon}
        groups = [g for g in self.mine[t] if not set(g[0]) & ending]
        if not groups:
            return
        pick = list(dict.fromkeys(groups[i % len(groups)] for i in picks))
        uuids = [u for g, _ in pick for u in g]
        excused = self._faults() > 0 or event is not None
        code, b = self.tc.call(self._racing(self.lc.remove("default", t, uuids, force=force),
                                            event, delay))
        self.steps.append(f"detach {t} {len(uuids)} GPU(s) force={force}"
                          f"{f' racing {event} +{delay * 1e3:g}ms' if event else ''} → {code}")
        self._answer(t, code, b if isinstance(b, dict) else {}, excused)
        if code == 200:
            for g in pick:
                self.mine[t].remove(g)
            for u in uuids:
                self.leases[t].pop(u, None)

    EVENTS = st.sampled_from(["container restart", "relist", "restart in relist",
                              "status churn", "worker restart"])

    @rule(t=st.sampled_from(TENANTS), n=st.integers(1, 2), entire=st.booleans(),
          event=EVENTS, delay=st.sampled_from([0.0, 0.001, 0.003]))
    def attach_racing(self, t, n, entire, event, delay):
        """An attach with a container restart, a relist or a worker restart in flight."""
        self._attach(t, n, entire, 0.0, (event, t), delay)

    @rule(t=st.sampled_from(TENANTS), picks=PICKS, event=EVENTS,
          delay=st.sampled_from([0.0, 0.001, 0.003]))
    def detach_racing(self, t, picks, event, delay):
        self._detach(t, False, picks, (event, t), delay)

    async def _racing(self, op, event, delay):
        if event is None:
            return await op
        task = asyncio.ensure_future(op)
        await asyncio.sleep(delay)
        what, t = event
        if what == "container restart":
            self.lc.cluster.restart_container("default", t, "main")
        elif what == "relist":
            self._expire()
        elif what == "restart in relist":     # the restart reaches the worker only by the relist
            self._expire()
            self.lc.cluster.restart_container("default", t, "main")
        elif what == "status churn":
            self._churn()
        else:
            await self.lc.stop_worker("node-0")
            w = await self.lc.start_worker("node-0")
            target = f"127.0.0.1:{w.grpc_port}"
            for _ in range(500):
                if self.lc.master.workers.target("node-0") == target:
                    break
                await asyncio.sleep(0.02)
        return await task

    @rule(seconds=st.sampled_from([0.2, 0.5]))
    def let_time_pass(self, seconds):
        self.steps.append(f"sleep {seconds}")
        time.sleep(seconds)

    @rule(t=st.sampled_from(TENANTS))
    def container_restart(self, t):
        self.steps.append(f"container restart {t}")
        self.tc.call(_sync(self.lc.cluster.restart_container, "default", t, "main"))

    @rule()
    def watch_relist(self):
        self.steps.append("watches expire (410): relist")
        self.tc.call(_sync(self._expire))

    @rule()
    def status_churn(self):
        """The kubelet updates every placeholder's status (a new resourceVersion each)."""
        self.steps.append("placeholder status churn")
        self.tc.call(_sync(self._churn))

    def _expire(self) -> None:
        expire = getattr(self.lc.cluster, "expire_watches", None)
        if expire is not None:         # an older fake without the hook: no relist
            expire()

    def _churn(self) -> None:
        c = self.lc.cluster
        for p in c.placeholders():
            pod = c.pods.get((p["metadata"]["namespace"], p["metadata"]["name"]))
            if pod is None:
                continue
            conds = pod.setdefault("status", {}).setdefault("conditions", [])
            conds[:] = [x for x in conds if x.get("type") != "GMChurn"] + [
                {"type": "GMChurn", "status": "True", "lastProbeTime": repr(time.time())}]
            c._bump("MODIFIED", pod)                               # noqa: SLF001

    @rule()
    def worker_restart(self):
        self.steps.append("worker restart")
        self.tc.call(self.lc.stop_worker("node-0"))
        w = self.tc.call(self.lc.start_worker("node-0"))
        target = f"127.0.0.1:{w.grpc_port}"
        self._until(lambda: self.lc.master.workers.target("node-0") == target, 10)

    @rule(n=st.integers(1, 3))
    def preemptor_arrives(self, n):
        """A Pod that outranks every tenant asks for ``n`` GPUs on the node, then goes away. It
        may get free GPUs, or (low pool class) preempt idle standbys; it must never preempt a
        placeholder that books a tenant's GPU — the invariant then sees the revocation."""
        c = self.lc.cluster
        name = f"hp-{len(self.steps)}"
        seen = c.preemptions

        def arrive():
            return c.create_pod("default", {
                "metadata": {"name": name},
                "spec": {"priorityClassName": "model-high",
                         "nodeSelector": {"kubernetes.io/hostname": "node-0"},
                         "containers": [{"name": "c", "image": "x:1", "resources": {
                             "limits": {"amd.com/gpu": str(n)}}}]}})
        hp = self.tc.call(_sync(arrive))
        self._until(lambda: podu.node_of(hp) or (podu.is_unschedulable(hp) and
                                                 not podu.nominated_node(hp)), 3)
        victims = c.victims[len(c.victims) - (c.preemptions - seen):] \
            if c.preemptions > seen else []
        self.steps.append(f"preemptor wants {n} → "
                          f"{'bound' if podu.node_of(hp) else 'pending'}, "
                          f"{len(victims)} victim(s)")
        booked = [v["metadata"]["name"] for v in victims
                  if (v["metadata"].get("labels") or {}).get("app") == "gpu-pool"
                  and (v["metadata"].get("annotations") or {}).get(MODE) != "standby"]
        check(not booked, f"placeholders of tenants preempted: {booked}; steps {self.steps}")
        self.tc.call(_sync(c.delete, "default", name, 0))

    @rule(faults=st.lists(st.tuples(st.sampled_from(["POST", "PATCH", "DELETE", "GET"]),
                                    st.booleans()), min_size=1, max_size=2))
    def lost_reply(self, faults):
        """The next request with each method on a pod fails: before it takes effect, or after
        it (the reply is lost). Whatever the next operations are, they must converge."""
        for method, after in faults:
            self.steps.append(f"next {method} fails {'after' if after else 'before'} applying")
            self.tc.call(_sync(self.lc.cluster.fail_next, method, 503, 1, after))

    @rule(method=st.sampled_from(["POST", "PATCH", "DELETE"]), after=st.booleans())
    def apiserver_outage(self, method, after):
        """The next five requests with a method on a pod fail — every retry of one request (a
        write that took effect with all its replies lost, when ``after``): the operation fails
        for good and must leave nothing behind that outlives its clean-up."""
        self.steps.append(f"next 5 {method}s fail {'after' if after else 'before'} applying")
        self.tc.call(_sync(self.lc.cluster.fail_next, method, 503, 5, after))

    # ------------------------------------------------------------------------ invariants
    async def _view(self):
        """(why not converged | None, {tenant: {uuid: (placeholder, lease_expires, entire)}})."""
        w = self._worker()
        svc = w.service
        out, hot_all = {}, []
        for t in TENANTS:
            pod = self.lc.cluster.get("default", t)
            issues = await self.lc.audit("default", t)
            if issues:
                return f"{t}: audit {[(i.kind, i.path) for i in issues][:3]}", {}
            st_ = await svc.pod_state(pod, fresh=True)
            if st_.mount_type.name == "UNKNOWN":
                return f"{t}: ledger unknown", {}
            raw = {p["metadata"]["name"]: p for p in svc.ph.owned_by(pod)}
            held = {}
            for ph in st_.placeholders:
                ann = (raw.get(ph.name) or {}).get("metadata", {}).get("annotations") or {}
                for g in st_.by_placeholder[(ph.namespace, ph.name)]:
                    held[g.uuid] = (ph.name, ann.get(LEASE), ann.get(MODE) == "entire")
            out[t] = held
            hot_all += list(held)
        phs = [p for p in self.lc.cluster.placeholders()
               if (p["metadata"].get("annotations") or {}).get(MODE) != "standby"]
        unbound = [p["metadata"]["name"] for p in phs if not p["spec"].get("nodeName")]
        if unbound:
            return f"unbound placeholders {unbound}", {}
        held_n = sum(int((p["metadata"].get("annotations") or {}).get(
            "gpumounter.amd.com/gpus") or 1) for p in phs)
        if len(hot_all) != len(set(hot_all)) or held_n != len(hot_all):
            return f"hot {sorted(hot_all)} vs placeholders holding {held_n}", {}
        return None, out

    @invariant()
    def converges_and_matches_the_clients(self):
        end = time.monotonic() + CONVERGE_S
        why, view = self.tc.call(self._view())
        while why is not None and time.monotonic() < end:
            time.sleep(0.05)
            why, view = self.tc.call(self._view())
        check(why is None, f"not converged after {CONVERGE_S}s: {why}; steps {self.steps}")
        now = time.monotonic()
        for t in TENANTS:
            held = view[t]
            # an expiry cannot land while the apiserver fails its writes: the slack runs from
            # the later of the lease's end and the last injected failure (an outage)
            up = self.lc.cluster.last_fault_at
            overdue = [u for u, (_, hi, _) in self.leases[t].items()
                       if now - max(hi, up) > SLACK]
            late = [u for u in overdue if u in held and held[u][0] == self.leases[t][u][2]
                    and (self.certain[t] or held[u][1])]
            check(not late, f"{t}: leases over more than {SLACK}s still attached: {late}; "
                            f"steps {self.steps}")
            for u in overdue:
                self.leases[t].pop(u)
            self.mine[t] = [g for g in self.mine[t] if not set(g[0]) & set(overdue)]
            fuzzy = {u for u, (lo, _, _) in self.leases[t].items() if lo <= now}
            if self.certain[t]:
                have = sorted(u for u in held if u not in fuzzy)
                want = sorted(u for g, _ in self.mine[t] for u in g if u not in fuzzy)
                check(have == want, f"{t}: ledger {have} != attached {want}; "
                                    f"steps {self.steps}")
            else:
                # after a failed request the client reads its state back from the ledger
                whole = tuple(u for u, h in held.items() if h[2])    # at most one entire mount
                self.mine[t] = [((u,), False) for u, h in held.items() if not h[2]] + \
                    ([(whole, True)] if whole else [])
                self.leases[t] = {u: e for u, e in self.leases[t].items()
                                  if u in held and held[u][0] == e[2] and held[u][1]}
                for u, (ph, exp, _) in held.items():
                    if exp and u not in self.leases[t]:
                        at = now + (float(exp) - time.time())
                        self.leases[t][u] = (at, at, ph)
                self.certain[t] = True


def _case(name: str, variant: dict):
    cls = type(name, (LedgerModel,), {"VARIANT": variant})
    case = cls.TestCase
    case.settings = settings(max_examples=EXAMPLES, stateful_step_count=STEPS, deadline=None,
                             suppress_health_check=list(HealthCheck), database=None,
                             phases=PHASES)
    return case


TestLedgerPlain = _case("LedgerPlain", {})
TestLedgerPool = _case("LedgerPool", {"worker_overrides": {"warm_pool_size": 2}})
TestLedgerDraPool = _case("LedgerDraPool", {"gpu_api": "dra",
                                            "worker_overrides": {"warm_pool_size": 2}})
TestLedgerTrimPool = _case("LedgerTrimPool", {"worker_overrides": {
    "warm_pool_size": 2, "placement_enforce": "trim"}})
# idle standbys preemptible (gpumounter-standby, value -10); attaches yield them
TestLedgerLowPool = _case("LedgerLowPool", {"worker_overrides": {
    "warm_pool_size": 2, "pool_priority_class": "gpumounter-standby"}})
# placeholders bound to the node at creation: the kubelet refuses those without room
TestLedgerDirectPool = _case("LedgerDirectPool", {"worker_overrides": {
    "warm_pool_size": 2, "placeholder_binding": "direct"}})
# a kubelet that frees a deleted Pod's devices 50 ms after the DELETE (admission refusals and
# re-bookings after every detach), with direct binding and a pool of preemptible standbys
TestLedgerTeardown = _case("LedgerTeardown", {
    "latency": LatencyModel(teardown_ms=50.0),
    "worker_overrides": {"warm_pool_size": 2, "placeholder_binding": "direct",
                         "pool_priority_class": "gpumounter-standby"}})
# the device manager's checkpoint keeps a deleted Pod until the next Allocate (a real kubelet's
# behaviour), with the teardown delay and a warm pool
TestLedgerLazyCheckpoint = _case("LedgerLazyCheckpoint", {
    "lazy_checkpoint": True, "latency": LatencyModel(teardown_ms=50.0),
    "worker_overrides": {"warm_pool_size": 2}})
