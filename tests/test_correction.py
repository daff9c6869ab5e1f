"""Placement correction (cluster/correction.py) against a fake apiserver whose every placeholder
POST, PATCH and DELETE may fail before it takes effect or after it (a lost reply).

State-level property test: for any node fragmentation, request size,
mount mode, device-plugin choice and fault schedule, the attach's outcome must satisfy

* safety — every GPU the correction returns (and the worker would mount) is booked by a
  placeholder that exists, is the owner's (no candidate mark) and holds exactly that GPU, before
  and after the reconciler's follow-up has run;
* no leak — once the follow-up has released what it was handed and the candidates no attach
  holds (worker/reconciler.py ``_react``/``_drop``), the owner's placeholders are exactly the
  returned ones (none when the attach failed).

The fake models what the real PlaceholderManager does under each fault (placeholder.py
``_create``/``_await_admission``/``release``/``confirm``): a created placeholder is scheduled and
given a GPU at once, whether or not its reply arrives; a DELETE whose reply is lost has happened.
The explicit example is the chaos finding fixed by 0b235e8 (an entire mount's second-round
release that took effect but lost its reply); this test fails on 0b235e8^.
"""
import asyncio
import types

import pytest
from hypothesis import HealthCheck, assume, example, given, settings
from hypothesis import strategies as s

from gpumounter_amd.cluster.placeholder import (InsufficientGPU, Placeholder, PlaceholderManager,
                                                Reservation, ReserveError)
from gpumounter_amd.utils.faults import FaultInjector, InjectedFault
from gpumounter_amd.utils.metrics import Metrics
from gpumounter_amd.worker.service import GpuMountService, PodGpuState

OWNER = {"metadata": {"name": "t", "namespace": "default", "uid": "uid-t"},
         "spec": {"nodeName": "node-0"}, "status": {"phase": "Running"}}


class FakeApi:
    """Placeholders of one owner on one node, with a fault per API call."""

    def __init__(self, inv, taken, policy, schedule):
        self.gpus = [g.index for g in inv.gpus()]
        self.bdf = {g.index: g.bdf for g in inv.gpus()}
        self.alloc = {i: "other" for i in taken}      # gpu index → holder uid
        self.pods = {}                                 # uid → {"gpus": [...], "candidate": bool}
        self.policy = policy
        self.schedule = list(schedule)
        self.stages = []           # stage faults around a release (FakePH.release)
        self.seq = 0
        self.calls = []

    def outcome(self, verb):
        o = self.schedule.pop(0) if self.schedule else "ok"
        self.calls.append((verb, o))
        return o

    def _schedule(self, uid, k):
        free = [i for i in self.gpus if i not in self.alloc]
        if len(free) < k:
            return None
        if self.policy == "last-free":
            free = free[::-1]
        elif self.policy.startswith("rot"):
            r = int(self.policy[3:]) % len(free)
            free = free[r:] + free[:r]
        got = free[:k]
        for i in got:
            self.alloc[i] = uid
        return got

    def create(self, k, candidate, faults=True):
        """POST → (placeholder or None, error or None). A created placeholder is admitted
        immediately (the scheduler binds, the plugin allocates) or stays unschedulable."""
        o = self.outcome("POST") if faults else "ok"
        if o == "before":
            return None, ReserveError("POST failed")
        self.seq += 1
        uid = f"ph{self.seq}"
        got = self._schedule(uid, k)
        self.pods[uid] = {"gpus": got, "candidate": candidate}
        if o == "after":
            return None, ReserveError("POST reply lost")
        ph = Placeholder("gpu-pool", f"t-slave-pod-{self.seq}", uid,
                         tuple(self.bdf[i] for i in got) if got else (),
                         "single", candidate)
        return ph, None

    def delete(self, uid):
        o = self.outcome("DELETE")
        if o == "before":
            return ReserveError("DELETE failed")
        p = self.pods.pop(uid, None)
        if p is not None:
            for i in p["gpus"] or ():
                self.alloc.pop(i, None)
        return ReserveError("DELETE reply lost") if o == "after" else None

    def patch_confirm(self, uid):
        o = self.outcome("PATCH")
        if o == "before":
            return ReserveError("PATCH failed")
        if uid in self.pods:
            self.pods[uid]["candidate"] = False
        return ReserveError("PATCH reply lost") if o == "after" else None


class FakePH:
    """The PlaceholderManager surface the correction uses, with its failure semantics."""

    def __init__(self, api):
        self.api = api
        self.device_ids = {}
        self.tombstones = {}
        self.keep_picked = PlaceholderManager.keep_picked

    async def release(self, phs):
        # the worker's stage fault around a release (faults "ledger_release"), as chaos injects
        # it: before any DELETE, or after every DELETE took effect
        stage = self.api.stages.pop(0) if self.api.stages else "ok"
        self.api.calls.append(("RELEASE", stage))
        if stage == "before":
            raise InjectedFault("injected fault at ledger_release (raise)")
        failed = []
        for p in phs:
            err = self.api.delete(p.uid)
            if err is not None:
                failed.append(p)
            else:
                self.device_ids.pop(p.uid, None)
        if failed:
            raise ReserveError(f"could not delete {len(failed)} placeholder(s)")
        if stage == "after":
            raise InjectedFault("injected fault at ledger_release (after)")

    async def hold_singles(self, owner, width, entire, group="", attach_id="", container="",
                           idempotency_key="", lease_expires=0.0):
        if width <= 0:
            return []
        created, errors = [], []
        for _ in range(width):
            ph, err = self.api.create(1, candidate=True)
            if ph is not None:
                created.append(ph)
            else:
                errors.append(err)
        if errors:
            await self.release(created)
            raise ReserveError(f"placeholder create failed: {errors[0]}")
        failed = [p for p in created if not p.device_ids]
        if failed:
            await self.release(failed)
        out = [p for p in created if p.device_ids]
        for p in out:
            self.device_ids[p.uid] = p.device_ids
        return out

    async def confirm(self, phs):
        todo = [p for p in phs if p.candidate]
        bad = []
        for p in todo:
            err = self.api.patch_confirm(p.uid)
            if err is None:
                p.candidate = False
            else:
                bad.append(err)
        if bad:
            raise ReserveError(f"confirming {len(bad)} placeholder(s) failed: {bad[0]}")


def make_service(inv, api):
    svc = GpuMountService.__new__(GpuMountService)
    svc.cfg = types.SimpleNamespace(topology_policy="xgmi", placement_enforce="auto")
    svc.inv = inv
    svc.ph = FakePH(api)
    svc.pool = None
    svc.faults = FaultInjector("")
    svc.metrics = Metrics()
    svc.unhealthy = set()
    svc.abandoned = {}
    svc.drops = []
    svc.followup = lambda ns, name, drop: svc.drops.append(list(drop))
    return svc


def follow_up(api, svc):
    """What the reconciler does next (worker/reconciler.py ``_react`` "followup" + sweep):
    release the handed placeholders that still exist, then every candidate of the owner. It
    retries with backoff until the apiserver answers, so it is run here without faults."""
    api.schedule = []
    for drop in svc.drops:
        for p in drop:
            if p.uid in api.pods:
                api.delete(p.uid)
    for uid in [u for u, p in api.pods.items() if p["candidate"]]:
        api.delete(uid)


def check_booked(api, out, n):
    got = 0
    for p in out.placeholders:
        live = api.pods.get(p.uid)
        assert live is not None, f"{p.name} is mounted but no longer exists"
        assert not live["candidate"], f"{p.name} is mounted but still a candidate"
        assert sorted(api.bdf[i] for i in live["gpus"]) == sorted(p.device_ids)
        got += len(p.device_ids)
    assert got == n


# taken GPUs, n, entire, plugin policy, fault schedule
SCENARIO = dict(taken=[0, 1, 2, 4, 5], n=2, entire=True, policy="first-free",
                schedule=["ok", "after"])


@pytest.fixture(scope="module")
def inv(mock_inventory):
    return mock_inventory


@settings(max_examples=400, deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.filter_too_much])
@given(taken=s.lists(s.integers(0, 7), max_size=6, unique=True),
       n=s.sampled_from([1, 2, 3, 4]), entire=s.booleans(),
       policy=s.sampled_from(["first-free", "last-free", "rot1", "rot2", "rot3", "rot5"]),
       schedule=s.lists(s.sampled_from(["ok", "ok", "before", "after"]), max_size=14),
       stages=s.lists(s.sampled_from(["ok", "ok", "before", "after"]), max_size=4))
@example(**SCENARIO, stages=[])
def test_correction_never_mounts_an_unbooked_gpu_and_leaks_nothing(inv, taken, n, entire,
                                                                  policy, schedule, stages):
    api = FakeApi(inv, taken, policy, schedule)
    api.stages = list(stages)
    assume(len(api.gpus) - len(taken) > n)         # else no other free GPU: nothing to correct
    svc = make_service(inv, api)
    # the plugin's admission of the attach itself (no faults: the correction's input)
    first, err = api.create(n if entire else 1, candidate=False, faults=False)
    phs = [first]
    for _ in range(0 if entire else n - 1):
        phs.append(api.create(1, candidate=False, faults=False)[0])
    res = Reservation(phs)
    ledger = {("x", f"other{i}"): [api.bdf[i]] for i in taken}
    st = PodGpuState(ledger=ledger)
    preferred = svc._preferred(n, st)               # placement's choice before reserving
    for p in phs:
        svc.ph.device_ids[p.uid] = p.device_ids     # admitted since the ledger view
    assume(svc._placement_worse(st, res.device_ids, preferred))  # else already best
    req = types.SimpleNamespace(is_entire_mount=entire, container="", idempotency_key="k")
    try:
        out = asyncio.run(svc._correct(OWNER, n, req, st, res))
    except (ReserveError, InsufficientGPU, InjectedFault):
        out = None
        # the attach failed: _add_gpu hands the pod to the follow-up as well
        svc.drops.append([])
    if out is not None:
        check_booked(api, out, n)
        assert not {p.uid for p in out.placeholders} & set(svc.abandoned)
    # until the follow-up has run, the owner's ledger view counts every live placeholder that
    # is neither a candidate nor handed over as abandoned: nothing beyond the answer may be one
    mine_now = {p.uid for p in out.placeholders} if out is not None else set()
    counted = [u for u, p in api.pods.items()
               if u not in mine_now and not p["candidate"] and u not in svc.abandoned]
    assert not counted, ("placeholders the owner's ledger counts beyond the answer",
                         counted, api.calls)
    follow_up(api, svc)
    mine = {p.uid for p in out.placeholders} if out is not None else set()
    assert set(api.pods) == mine, (api.calls, api.pods, mine)
    if out is not None:
        check_booked(api, out, n)                   # the follow-up took none of them


def test_the_lost_reply_scenario_reaches_the_second_round(inv):
    """The explicit example does exercise the second round (it is not vacuous)."""
    api = FakeApi(inv, **{k: SCENARIO[k] for k in ("taken", "policy", "schedule")})
    svc = make_service(inv, api)
    first, _ = api.create(2, candidate=False, faults=False)
    req = types.SimpleNamespace(is_entire_mount=True, container="", idempotency_key="k")
    st = PodGpuState(ledger={("x", f"o{i}"): [api.bdf[i]] for i in SCENARIO["taken"]})
    assert svc._placement_worse(st, first.device_ids, svc._preferred(2, st))
    svc.ph.device_ids[first.uid] = first.device_ids
    with pytest.raises((ReserveError, InsufficientGPU)):
        asyncio.run(svc._correct(OWNER, 2, req, st, Reservation([first])))
    assert ("DELETE", "after") in api.calls


class LaggingApi(FakeApi):
    """The kubelet frees a deleted placeholder's devices ``lag_s`` after the DELETE (it acts on
    its own watch of the deletion): a re-hold sent earlier finds them still booked."""

    def __init__(self, *a, lag_s=0.3, **k):
        super().__init__(*a, **k)
        self.lag_s = lag_s
        self.freed_at = {}          # gpu index → monotonic time it becomes allocatable

    def delete(self, uid):
        import time

        p = self.pods.get(uid)
        err = super().delete(uid)
        if p is not None and uid not in self.pods:
            for i in p["gpus"] or ():
                self.freed_at[i] = time.monotonic() + self.lag_s
        return err

    def _schedule(self, uid, k):
        import time

        now = time.monotonic()
        lagging = {i for i, t in self.freed_at.items() if t > now}
        free = [i for i in self.gpus if i not in self.alloc and i not in lagging]
        if len(free) < k:
            return None
        saved = self.alloc
        self.alloc = {**saved, **{i: "lag" for i in lagging}}
        try:
            got = super()._schedule(uid, k)
        finally:
            for i in lagging:
                self.alloc.pop(i, None)
            self.alloc.update({i: uid for i in got or ()})
        return got


def test_second_round_outlasts_a_slow_kubelet_release(inv):
    """the second round of an entire-mount correction re-holds GPUs it just let go.
    With the kubelet 0.3 s behind the DELETE, the round-5 retry budget (0, 50, 200 ms) gave up
    and the attach kept the worse placement; the re-hold now outlasts the lag and the
    correction lands on the best set."""
    from gpumounter_amd.cluster.correction import Correction

    api = LaggingApi(inv, SCENARIO["taken"], SCENARIO["policy"], [], lag_s=0.3)
    svc = make_service(inv, api)
    first, _ = api.create(2, candidate=False, faults=False)
    req = types.SimpleNamespace(is_entire_mount=True, container="", idempotency_key="k")
    st = PodGpuState(ledger={("x", f"o{i}"): [api.bdf[i]] for i in SCENARIO["taken"]})
    best = svc._preferred(2, st)
    assert svc._placement_worse(st, first.device_ids, best)
    svc.ph.device_ids[first.uid] = first.device_ids
    out = asyncio.run(svc._correct(OWNER, 2, req, st, Reservation([first])))
    assert sorted(out.device_ids) == sorted(best), (out.device_ids, best, api.calls)
    check_booked(api, out, 2)
    # the round-5 budget is not enough for this kubelet
    old = Correction.REHOLD_DELAYS_S
    try:
        Correction.REHOLD_DELAYS_S = (0.0, 0.05, 0.2)
        api2 = LaggingApi(inv, SCENARIO["taken"], SCENARIO["policy"], [], lag_s=0.3)
        svc2 = make_service(inv, api2)
        first2, _ = api2.create(2, candidate=False, faults=False)
        svc2.ph.device_ids[first2.uid] = first2.device_ids
        try:
            out2 = asyncio.run(svc2._correct(OWNER, 2, req, st, Reservation([first2])))
            assert sorted(out2.device_ids) != sorted(best)
        except (ReserveError, InsufficientGPU):
            pass
    finally:
        Correction.REHOLD_DELAYS_S = old
