"""Warm-pool hand-offs (cluster/pool.py) against an apiserver whose every GET/PATCH/DELETE may
fail before it takes effect or after it, seen by two worker incarnations whose caches lag the
apiserver independently (a relist, a killed worker's requests still in flight).

State-level property: for any sequence of claims, give-backs and cache catch-ups and any fault
schedule,

* a claim answered with placeholders is the only holder of each of them: no placeholder is
  held by two claims at once;
* every placeholder a claim holds is, at the apiserver, owned by that claim's Pod until the
  claim gives it back;
* a give-back never changes the owner of a placeholder some other claim holds;
* a claim refused without an error leaves none of its placeholders claimed, and a give-back
  that returns leaves none of them with the Pod that gave them back.

The explicit example is the chaos finding of round 4 (`profiles/r4_chaos_full/`): the second
incarnation's cache still shows a placeholder as standby after the first one claimed it. With
unconditional claim PATCHes both claims succeed; this test fails on that code.
"""
import asyncio
import copy

import pytest
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as s

from gpumounter_amd.cluster.kube import ApiError, Conflict, NotFound
from gpumounter_amd.cluster.placeholder import (STANDBY_PREFIX, PlaceholderManager,
                                                ReserveError)
from gpumounter_amd.cluster.pool import WarmPool
from gpumounter_amd.models.types import (ANN_MOUNT_MODE, ANN_OWNER_UID, LABEL_APP,
                                         LABEL_APP_VALUE, MODE_STANDBY)
from gpumounter_amd.utils.config import Config

NS = "gpu-pool"


def merge(target, patch):
    for k, v in patch.items():
        if v is None:
            target.pop(k, None)
        elif isinstance(v, dict):
            target[k] = merge(dict(target.get(k) or {}), v)
        else:
            target[k] = v
    return target


class FakeKube:
    """Pods of the pool namespace with resourceVersions and preconditions. Each call's outcome
    comes from the schedule, as the KubeClient (with its retries) would see it: ``ok``;
    ``before`` (every attempt failed, nothing applied); ``after`` (applied, the reply lost,
    the retry answered as a fresh request: a conditional one meets its own change as a
    conflict); ``lost`` (applied, every reply lost)."""

    def __init__(self, schedule):
        self.pods = {}
        self.rv = 100
        self.schedule = list(schedule)

    def outcome(self):
        return self.schedule.pop(0) if self.schedule else "ok"

    def add(self, name, uid):
        self.rv += 1
        self.pods[name] = {"metadata": {
            "namespace": NS, "name": name, "uid": uid, "resourceVersion": str(self.rv),
            "labels": {LABEL_APP: LABEL_APP_VALUE, "gpumounter.amd.com/node": "node-0"},
            "annotations": {ANN_MOUNT_MODE: MODE_STANDBY, "gpumounter.amd.com/gpus": "1"}},
            "spec": {"nodeName": "node-0"}, "status": {"phase": "Running"}}

    async def get_pod(self, ns, name):
        await asyncio.sleep(0)
        if self.outcome() == "before":
            raise ApiError(503, "injected")
        if name not in self.pods:
            raise NotFound(404, name)
        return copy.deepcopy(self.pods[name])

    def _apply_patch(self, name, patch):
        pod = self.pods.get(name)
        if pod is None:
            raise NotFound(404, name)
        md = dict(patch.get("metadata") or {})
        want = md.pop("resourceVersion", None)
        if want is not None and want != pod["metadata"]["resourceVersion"]:
            raise Conflict(409, "modified")
        merge(pod["metadata"], md)
        self.rv += 1
        pod["metadata"]["resourceVersion"] = str(self.rv)
        return copy.deepcopy(pod)

    async def patch_pod(self, ns, name, patch):
        await asyncio.sleep(0)
        o = self.outcome()
        if o == "before":
            raise ApiError(503, "injected")
        out = self._apply_patch(name, patch)
        if o == "lost":
            raise ApiError(503, "reply lost")
        if o == "after":
            return self._apply_patch(name, patch)      # the client's retry
        return out

    def _apply_delete(self, name, uid, rv):
        pod = self.pods.get(name)
        if pod is None:
            raise NotFound(404, name)
        if (uid and pod["metadata"]["uid"] != uid) or \
                (rv and pod["metadata"]["resourceVersion"] != rv):
            raise Conflict(409, "precondition")
        return self.pods.pop(name)

    async def delete_pod(self, ns, name, grace_period_s=None, uid="", resource_version=""):
        await asyncio.sleep(0)
        o = self.outcome()
        if o == "before":
            raise ApiError(503, "injected")
        out = self._apply_delete(name, uid, resource_version)
        if o == "lost":
            raise ApiError(503, "reply lost")
        if o == "after":
            return self._apply_delete(name, uid, resource_version)
        return out


class FakeInformer:
    """A cache that catches up with the apiserver only when told to (``sync``)."""

    def __init__(self, kube):
        self.kube = kube
        self.cache = {}
        self.epoch = 0
        self.handlers = []

    def sync(self):
        self.cache = {(NS, n): copy.deepcopy(p) for n, p in self.kube.pods.items()}
        self.epoch += 1

    def upsert(self, pod, epoch=None):
        if epoch is not None and epoch != self.epoch:
            return                              # a relist came between: dropped (the bug's cause)
        md = pod["metadata"]
        self.cache[(md["namespace"], md["name"])] = copy.deepcopy(pod)

    def list(self, pred=lambda p: True):
        return [p for p in self.cache.values() if pred(p)]

    async def poke(self):
        pass


def incarnation(kube, inv, bdfs):
    cfg = Config(warm_pool_size=8, pool_namespace=NS, topology_policy="xgmi")
    inf = FakeInformer(kube)
    ph = PlaceholderManager(cfg, kube, None, inf, "node-0")
    for name, p in kube.pods.items():
        ph.device_ids[p["metadata"]["uid"]] = (bdfs[name],)
    inf.sync()
    return WarmPool(cfg, ph, inv)


OUTCOMES = s.sampled_from(["ok", "ok", "ok", "before", "after", "lost"])
OPS = s.lists(s.one_of(
    s.tuples(s.just("claim"), s.integers(0, 1), s.integers(0, 2), s.integers(1, 2)),
    s.tuples(s.just("give_back"), s.integers(0, 1), s.integers(0, 2), s.just(0)),
    s.tuples(s.just("sync"), s.integers(0, 1), s.just(0), s.just(0)),
    s.tuples(s.just("relist"), s.integers(0, 1), s.just(0), s.just(0))), min_size=1, max_size=12)

# the chaos finding: incarnation 1's cache is behind incarnation 0's claim of the only standby
SCENARIO = {"ops": [("claim", 0, 0, 1), ("claim", 1, 1, 1)], "schedule": []}
# a claim PATCH applied behind a lost reply, then the undo's read fails: the placeholder is
# deleted as this attach's stray, which must not be mistaken for someone else's
STRAY = {"ops": [("claim", 0, 0, 1)], "schedule": ["lost", "before"]}
# the same Pod claims through a stale cache what its earlier attach holds, and every read after
# the conflict fails: the failed attach's clean-up must not delete the earlier attach's claim
SAME_POD = {"ops": [("claim", 0, 0, 1), ("claim", 1, 0, 1)], "schedule": ["ok", "before", "before"]}


def run_scenario(inv, ops, schedule):
    kube = FakeKube([])
    gpus = inv.gpus()[:3]
    bdfs = {}
    for i, g in enumerate(gpus):
        name = f"{STANDBY_PREFIX}node-0-{i:04d}"
        kube.add(name, f"uid-sb{i}")
        bdfs[name] = g.bdf
    pools = [incarnation(kube, inv, bdfs), incarnation(kube, inv, bdfs)]
    kube.schedule = list(schedule)
    owners = [{"metadata": {"name": f"t{i}", "namespace": "default", "uid": f"uid-t{i}"},
               "spec": {"nodeName": "node-0"}} for i in range(3)]
    held = {}                      # placeholder name → (owner index, pool index)
    problems = []

    async def main():
        for step, (op, pi, oi, n) in enumerate(ops):
            pool = pools[pi]
            if op == "sync":
                pool.ph.informer.sync()
            elif op == "relist":
                pool.ph.informer.epoch += 1          # in-flight write-throughs are dropped
            elif op == "claim":
                try:
                    res = await pool.claim(owners[oi], n, False, [], attach_id=f"add-{step}")
                except (ApiError, ReserveError):
                    res = False         # failed: the worker's follow-up cleans up after it
                if res is None:         # refused cleanly: nothing of this attach stays claimed
                    left = [nm for nm, p in kube.pods.items()
                            if (p["metadata"].get("annotations") or {}).get(
                                "gpumounter.amd.com/attach-id") == f"add-{step}"]
                    if left:
                        problems.append(f"step {step}: claim refused but {left} stay claimed "
                                        f"by t{oi}")
                for ph in (res.placeholders if res else []):
                    if ph.name in held:
                        problems.append(f"step {step}: {ph.name} claimed by t{oi} while t"
                                        f"{held[ph.name][0]} holds it")
                    held[ph.name] = (oi, pi)
            elif op == "give_back":
                mine = [n_ for n_, (o, p) in held.items() if o == oi and p == pi]
                phs = []
                for name in mine:
                    c = pool.ph.informer.cache.get((NS, name))
                    ph = pool.ph.cached(c) if c is not None else None
                    if ph is None:
                        continue
                    ph.owner_uid = owners[oi]["metadata"]["uid"]
                    phs.append(ph)
                    del held[name]
                if phs:
                    try:
                        await pool.give_back(phs)
                    except (ApiError, ReserveError):
                        continue        # failed: the worker's follow-up retries the release
                    mine_left = [ph.name for ph in phs if (
                        (kube.pods.get(ph.name) or {}).get("metadata", {}).get(
                            "annotations") or {}).get(ANN_OWNER_UID) == ph.owner_uid]
                    if mine_left:
                        problems.append(f"step {step}: t{oi} gave back {mine_left} and still "
                                        f"owns them")
            for name, (o, _) in held.items():
                pod = kube.pods.get(name)
                got = ((pod or {}).get("metadata", {}).get("annotations") or {}).get(ANN_OWNER_UID)
                if got != owners[o]["metadata"]["uid"]:
                    problems.append(f"step {step} ({op}): {name} held by t{o}, owner at the "
                                    f"apiserver {got!r}")
    asyncio.run(main())
    return problems


@pytest.fixture(scope="module")
def inv(mock_inventory):
    return mock_inventory


@settings(max_examples=300, deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(ops=OPS, schedule=s.lists(OUTCOMES, max_size=20))
@example(**SCENARIO)
@example(**STRAY)
@example(**SAME_POD)
def test_a_standby_placeholder_is_never_held_by_two_claims(inv, ops, schedule):
    problems = run_scenario(inv, ops, schedule)
    assert not problems, problems[:3]
