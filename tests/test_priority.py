"""Placeholder priority and preemption (cluster/placeholder.py ``priority_for``, cluster/pool.py
``yield_low``, fakes/apiserver.py's Priority admission and preemption).

The reference's slave pods carry no priority (reference:
pkg/util/gpu/allocator/allocator.go:189-234): on a full node, any higher-priority Pod that asks
for a GPU makes the scheduler preempt a slave pod, and the GPU goes back to the scheduler while
its tenant still uses it. Under the shipped deploy a placeholder never ranks below its tenant
and never preempts; a low pool class keeps only *idle* standbys preemptible."""
import asyncio
import time

import pytest

from gpumounter_amd.cluster.pool import is_standby
from gpumounter_amd.fakes.apiserver import FakeCluster
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.models import pod as podu


def _preemptor(lc, name: str, gpus: int = 1, cls: str = "high") -> dict:
    return lc.cluster.create_pod("default", {
        "metadata": {"name": name},
        "spec": {"priorityClassName": cls, "nodeSelector": {"kubernetes.io/hostname": "node-0"},
                 "containers": [{"name": "c", "image": "x:1",
                                 "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]}})


async def _until(pred, timeout: float = 5.0, what: str = "") -> None:
    end = time.monotonic() + timeout
    while not pred():
        assert time.monotonic() < end, f"timed out waiting for {what or pred}"
        await asyncio.sleep(0.01)


def _held_by(lc, t: str):
    return [p for p in lc.cluster.placeholders()
            if (p["metadata"].get("annotations") or {}).get("gpumounter.amd.com/owner-name") == t
            and not is_standby(p)]


def test_full_node_higher_priority_pod_stays_pending_under_the_default_deploy():
    async def main():
        async with LocalCluster() as lc:
            lc.cluster.add_priority_class("high", 1000)
            lc.tenant("t")
            code, b = await lc.add("default", "t", 8)
            assert code == 200 and len(b["devices"]) == 8
            phs = _held_by(lc, "t")
            assert {p["spec"]["priorityClassName"] for p in phs} == {"gpumounter-placeholder"}
            assert {p["spec"]["priority"] for p in phs} == {1000000}
            assert {p["spec"]["preemptionPolicy"] for p in phs} == {"Never"}
            hp = _preemptor(lc, "hp")
            await _until(lambda: podu.is_unschedulable(hp), what="hp unschedulable")
            await asyncio.sleep(0.3)                     # retries on freed capacity: none
            assert podu.is_unschedulable(hp) and not podu.node_of(hp)
            assert not podu.nominated_node(hp) and lc.cluster.preemptions == 0
            assert "no lower-priority victims" in podu.is_unschedulable(hp)
            assert len(_held_by(lc, "t")) == 8 and not await lc.audit("default", "t")
            # the hot-mounted GPUs are still the tenant's: it can remove them as usual
            code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]][:1])
            assert code == 200
            # ... and the freed GPU goes to the pending Pod
            await _until(lambda: podu.node_of(hp) == "node-0", what="hp bound")
    asyncio.run(main())


def test_without_a_floor_class_the_reference_hazard_is_real():
    """placeholder_priority_class="" with a tenant of default priority: placeholders rank 0
    (as the reference's slave pods), the scheduler preempts one for a priority-1000 Pod, and
    the worker must revoke that GPU from the running tenant. This is the failure the default
    deploy prevents (test above)."""
    async def main():
        async with LocalCluster(worker_overrides={"placeholder_priority_class": ""}) as lc:
            lc.cluster.add_priority_class("high", 1000)
            lc.tenant("t")
            code, b = await lc.add("default", "t", 8)
            assert code == 200
            assert {p["spec"].get("priority") for p in _held_by(lc, "t")} == {0}
            hp = _preemptor(lc, "hp")
            await _until(lambda: podu.node_of(hp) == "node-0", what="hp bound by preemption")
            assert lc.cluster.preemptions == 1
            await _until(lambda: len(_held_by(lc, "t")) == 7, what="revocation")
            st = await lc.nodes["node-0"].worker.service.pod_state(
                lc.cluster.get("default", "t"), fresh=True)
            assert len(st.hot) == 7
            await _until(lambda: any(e.get("reason") == "GPURevoked" for e in
                                     lc.cluster.events_for("default", "t")), what="event")
            ev = next(e for e in lc.cluster.events_for("default", "t")
                      if e.get("reason") == "GPURevoked")
            assert "preempted by the scheduler" in ev["message"]
    asyncio.run(main())


def test_tenant_above_the_floor_gets_its_own_class():
    async def main():
        async with LocalCluster() as lc:
            lc.cluster.add_priority_class("critical-tenant", 5000000)
            pod = lc.cluster.create_running_pod("default", {
                "metadata": {"name": "vip"},
                "spec": {"priorityClassName": "critical-tenant",
                         "containers": [{"name": "main", "image": "x:1"}]}}, "node-0")
            assert pod["spec"]["priority"] == 5000000
            code, _ = await lc.add("default", "vip", 2)
            assert code == 200
            phs = _held_by(lc, "vip")
            assert {p["spec"]["priorityClassName"] for p in phs} == {"critical-tenant"}
            assert {p["spec"]["priority"] for p in phs} == {5000000}
    asyncio.run(main())


def test_missing_floor_class_falls_back_to_the_tenants_class():
    async def main():
        async with LocalCluster(priority_classes=False) as lc:
            lc.cluster.add_priority_class("team", 300)
            lc.cluster.create_running_pod("default", {
                "metadata": {"name": "t"},
                "spec": {"priorityClassName": "team",
                         "containers": [{"name": "main", "image": "x:1"}]}}, "node-0")
            ph = lc.nodes["node-0"].worker.placeholders
            assert ph.class_values == {"gpumounter-placeholder": None}
            code, _ = await lc.add("default", "t", 1)
            assert code == 200
            (p,) = _held_by(lc, "t")
            assert p["spec"]["priorityClassName"] == "team" and p["spec"]["priority"] == 300
    asyncio.run(main())


def test_class_deleted_after_start_is_handled_at_create_time():
    async def main():
        async with LocalCluster() as lc:
            lc.cluster.priority_classes.pop("gpumounter-placeholder")
            lc.tenant("t")
            code, _ = await lc.add("default", "t", 1)
            assert code == 200
            ph = lc.nodes["node-0"].worker.placeholders
            assert ph.class_values["gpumounter-placeholder"] is None
            assert ph.priority_fallbacks == 1
            code, _ = await lc.add("default", "t", 1)        # now created without a retry
            assert code == 200 and ph.priority_fallbacks == 1
    asyncio.run(main())


def test_low_pool_class_standbys_are_preemptible_claims_rebook_and_the_pool_refills():
    async def main():
        ov = {"warm_pool_size": 2, "pool_priority_class": "gpumounter-standby"}
        async with LocalCluster(worker_overrides=ov) as lc:
            lc.cluster.add_priority_class("high", 1000)
            pool = lc.nodes["node-0"].worker.pool
            await _until(lambda: len(pool.standby()) == 2, what="pool filled")
            assert {p.priority for p in pool.standby()} == {-10}
            lc.tenant("a")
            lc.tenant("b")
            # 6 GPUs for a: the standbys rank below a's placeholders, so a books free GPUs
            code, b_a = await lc.add("default", "a", 6)
            assert code == 200 and len(pool.standby()) == 2
            assert {p["spec"]["priority"] for p in _held_by(lc, "a")} == {1000000}
            # the node is full (6 hot + 2 standby): a priority-1000 Pod preempts one *standby*
            hp = _preemptor(lc, "hp")
            await _until(lambda: podu.node_of(hp) == "node-0", what="hp bound")
            assert lc.cluster.preemptions == 1 and len(_held_by(lc, "a")) == 6
            await _until(lambda: len(pool.standby()) == 1, what="one standby left")
            # b's attach yields the last standby and books its GPU at b's rank
            code, b_b = await lc.add("default", "b", 1)
            assert code == 200, b_b
            (p,) = _held_by(lc, "b")
            assert p["spec"]["priority"] == 1000000
            assert not await lc.audit("default", "a") and not await lc.audit("default", "b")
            assert pool.standby() == []
            # capacity frees (the preemptor ends): the pool refills from it
            lc.cluster.delete("default", "hp", grace=0)
            await _until(lambda: len(pool.standby()) == 1, 10, what="pool refilled")
            assert {p.priority for p in pool.standby()} == {-10}
            # a detached tenant placeholder does not become a (non-preemptible) standby
            code, _ = await lc.remove("default", "b", [d["uuid"] for d in b_b["devices"]])
            assert code == 200
            await _until(lambda: len(pool.standby()) == 2, 10, what="pool refilled to 2")
            assert {p.priority for p in pool.standby()} == {-10}
    asyncio.run(main())


def test_default_pool_standbys_are_not_preemptible_and_claims_stay_a_patch():
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 2}) as lc:
            lc.cluster.add_priority_class("high", 1000)
            pool = lc.nodes["node-0"].worker.pool
            await _until(lambda: len(pool.standby()) == 2, what="pool filled")
            assert {p.priority for p in pool.standby()} == {1000000}
            lc.tenant("a")
            code, _ = await lc.add("default", "a", 6)
            assert code == 200
            await _until(lambda: len(pool.standby()) == 2, what="pool refilled")
            hp = _preemptor(lc, "hp")
            await _until(lambda: podu.is_unschedulable(hp), what="hp unschedulable")
            await asyncio.sleep(0.2)
            assert lc.cluster.preemptions == 0 and len(pool.standby()) == 2
            lc.tenant("b")
            posts = lc.cluster.requests_by_verb.get("POST", 0)
            code, b = await lc.add("default", "b", 1)
            assert code == 200
            assert {t["name"] for t in b["timings"]} >= {"pool_claim"}
            assert lc.cluster.requests_by_verb.get("POST", 0) == posts   # no placeholder create
    asyncio.run(main())


# ---------------------------------------------------------------------- the fake's own model
def test_fake_priority_admission_matches_the_admission_plugin():
    c = FakeCluster()
    c.add_priority_class("p", 7, "Never")
    pod = c.create_pod("ns", {"metadata": {"name": "a"}, "spec": {"priorityClassName": "p"}},
                       schedule=False)
    assert pod["spec"]["priority"] == 7 and pod["spec"]["preemptionPolicy"] == "Never"
    for spec, msg in (({"priorityClassName": "nope"}, "no PriorityClass with name nope"),
                      ({"priorityClassName": "p", "priority": 8}, "integer value of priority"),
                      ({"priorityClassName": "p", "preemptionPolicy": "PreemptLowerPriority"},
                       "PreemptionPolicy")):
        with pytest.raises(Exception) as ei:
            c.create_pod("ns", {"metadata": {"name": "b"}, "spec": spec}, schedule=False)
        assert ei.value.status == 403 and msg in ei.value.text
    c.add_priority_class("dflt", 5, global_default=True)
    pod = c.create_pod("ns", {"metadata": {"name": "c"}, "spec": {}}, schedule=False)
    assert pod["spec"]["priorityClassName"] == "dflt" and pod["spec"]["priority"] == 5


def test_fake_scheduler_keeps_a_preemptors_room_for_it():
    """A preemption nominates the node; a lower-priority Pod created while the victims
    terminate cannot take the room back (kube-scheduler's nominated-pod accounting)."""
    async def main():
        async with LocalCluster(start_master=False, start_workers=False) as lc:
            c = lc.cluster
            c.add_priority_class("low", 1)
            c.add_priority_class("high", 1000)
            for i in range(8):
                p = _preemptor(lc, f"low{i}", 1, "low")
                p["spec"]["terminationGracePeriodSeconds"] = 1
            await _until(lambda: all(podu.node_of(c.get("default", f"low{i}")) for i in range(8)))
            for i in range(8):              # running, so deletion waits for their grace
                c.get("default", f"low{i}")["status"]["phase"] = "Running"
            c.latency.stop_ms = 200.0
            hp = _preemptor(lc, "hp", 2, "high")
            await _until(lambda: podu.nominated_node(hp) == "node-0", what="nomination")
            late = _preemptor(lc, "late", 1, "low")
            await _until(lambda: podu.node_of(hp) == "node-0", 5, what="hp bound")
            assert c.preemptions == 2 and not podu.node_of(late)
    asyncio.run(main())


def test_attach_during_a_low_refill_cancels_it_instead_of_racing_it():
    """Right after a detach the pool refills with a low standby; an attach at tenant rank that
    arrives while that standby is being admitted cannot claim it, and would lose the last free
    GPU to it (then wait for its admission, yield it and book again: two admissions). The
    pending standby is cancelled first: one admission."""
    from gpumounter_amd.fakes.apiserver import LatencyModel

    async def main():
        ov = {"warm_pool_size": 1, "pool_priority_class": "gpumounter-standby"}
        lat = LatencyModel(schedule_ms=100.0, admit_ms=100.0)
        async with LocalCluster(worker_overrides=ov, latency=lat) as lc:
            pool = lc.nodes["node-0"].worker.pool
            lc.tenant("a")
            lc.tenant("b")
            code, _ = await lc.add("default", "a", 7)          # 7 booked, 1 left for the pool
            assert code == 200
            await _until(lambda: len(pool.standby()) == 1, 10, what="pool filled")
            code, b1 = await lc.add("default", "b", 1)         # yields the standby
            assert code == 200
            code, _ = await lc.remove("default", "b", [d["uuid"] for d in b1["devices"]])
            assert code == 200
            await _until(lambda: pool.refilling(), 5, what="refill in flight")
            t0 = time.monotonic()
            code, b2 = await lc.add("default", "b", 1)
            took = time.monotonic() - t0
            assert code == 200, b2
            assert took < 0.33, took                           # one admission (0.2 s), not two
            assert not await lc.audit("default", "b")
    asyncio.run(main())
