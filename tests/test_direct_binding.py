"""placeholder_binding=direct (cluster/placeholder.py ``build``, fakes/apiserver.py ``_schedule``):
placeholders are created with spec.nodeName, so the kubelet admits them without a scheduling
cycle; the kubelet's own admission refuses one the node has no room for (OutOfamd.com/gpu),
which the attach reports as the reference's insufficient-GPU answer and cleans up.
The reference's slave pods always go through kube-scheduler (allocator.go:189-234)."""
import asyncio
import time

import pytest

from gpumounter_amd.cluster.pool import is_standby
from gpumounter_amd.fakes.apiserver import LatencyModel
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.utils.config import Config

SLOW_SCHEDULER = LatencyModel(schedule_ms=400.0)
DIRECT = {"placeholder_binding": "direct"}


def _attach_ms(binding: dict) -> float:
    async def main():
        async with LocalCluster(latency=SLOW_SCHEDULER, worker_overrides=binding) as lc:
            lc.tenant("t")
            t0 = time.perf_counter()
            code, b = await lc.add("default", "t", 2)
            ms = (time.perf_counter() - t0) * 1e3
            assert code == 200 and len(b["devices"]) == 2, b
            phs = [p for p in lc.cluster.placeholders() if not is_standby(p)]
            assert phs and all(p["spec"].get("nodeName") == "node-0" for p in phs)
            if binding:
                assert all(p["spec"]["nodeName"] == "node-0" and
                           p["spec"].get("priorityClassName") == "gpumounter-placeholder"
                           for p in phs)
            assert not await lc.audit("default", "t")
            code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
            assert code == 200
            return ms
    return asyncio.run(main())


def test_direct_binding_skips_the_scheduling_cycle():
    assert _attach_ms({}) >= 400.0            # the scheduler's cycle is on the attach path
    assert _attach_ms(DIRECT) < 300.0         # ... and not with direct binding


def test_direct_binding_on_a_full_node_is_refused_by_the_kubelet_and_cleaned_up():
    async def main():
        async with LocalCluster(worker_overrides=DIRECT) as lc:
            lc.tenant("a")
            lc.tenant("b")
            code, _ = await lc.add("default", "a", 6)
            assert code == 200
            code, body = await lc.add("default", "b", 4)
            assert code == 500 and "Insufficient GPU" in str(body), body
            # the refused placeholder is not left behind (Failed Pods are not garbage
            # collected on their own)
            end = time.monotonic() + 5
            while any((p["metadata"].get("annotations") or {})
                      .get("gpumounter.amd.com/owner-name") == "b"
                      for p in lc.cluster.placeholders()):
                assert time.monotonic() < end, "refused placeholder left behind"
                await asyncio.sleep(0.02)
            code, b = await lc.add("default", "b", 2)
            assert code == 200 and len(b["devices"]) == 2
            assert not await lc.audit("default", "a") and not await lc.audit("default", "b")
    asyncio.run(main())


def test_direct_binding_fills_the_warm_pool():
    async def main():
        async with LocalCluster(worker_overrides={**DIRECT, "warm_pool_size": 2}) as lc:
            lc.tenant("t")
            pool = lc.nodes["node-0"].worker.pool
            end = time.monotonic() + 5
            while len(pool.standby()) < 2:
                assert time.monotonic() < end, "pool not filled"
                await asyncio.sleep(0.02)
            assert all(p["spec"].get("nodeName") == "node-0"
                       for p in lc.cluster.placeholders() if is_standby(p))
            code, b = await lc.add("default", "t", 1)
            assert code == 200 and b["devices"]
    asyncio.run(main())


def test_direct_binding_is_refused_with_dra():
    with pytest.raises(ValueError, match="placeholder_binding"):
        Config().replace(gpu_allocation="dra", placeholder_binding="direct")


def _failed(lc, body: dict) -> dict:
    """``body`` created and refused at admission, as the kubelet refuses a directly bound Pod
    on a full node (its worker died before it could delete it)."""
    pod = lc.cluster.create_pod(body["metadata"]["namespace"], body, schedule=False)
    pod["status"].update(phase="Failed", reason="OutOfamd.com/gpu")
    lc.cluster._bump("MODIFIED", pod)              # noqa: SLF001 - the watch event
    return pod


def test_placeholders_refused_at_admission_are_released_at_once():
    """A Failed placeholder (or standby) holds no device and never runs: the sweep releases
    an owner's at once (not after stuck_after_s), the pool's refill its own — a Failed standby
    counted as pending would keep the pool from refilling for good."""
    async def main():
        async with LocalCluster(worker_overrides={**DIRECT, "warm_pool_size": 1}) as lc:
            w = lc.nodes["node-0"].worker
            owner = lc.tenant("t")
            code, _ = await lc.add("default", "t", 1)
            assert code == 200
            ph = _failed(lc, w.service.ph.build(owner, 1, "single"))
            sb = _failed(lc, w.pool.standby_body())
            await asyncio.sleep(0.05)
            assert w.pool.pending() == 0            # refused, not being admitted
            rep = await w.reconciler.run_once()
            assert ph["metadata"]["name"] in rep.stuck
            await w.pool.refill()
            names = {p["metadata"]["name"] for p in lc.cluster.placeholders()}
            assert ph["metadata"]["name"] not in names and sb["metadata"]["name"] not in names
            assert not await lc.audit("default", "t")
    asyncio.run(main())



@pytest.mark.parametrize("binding", [{}, DIRECT], ids=["scheduler", "direct"])
def test_an_attach_right_after_a_detach_outlasts_the_kubelets_teardown(binding):
    """The kubelet frees a deleted Pod's devices only once it has stopped it (here 150 ms after
    the DELETE's answer). The scheduler, and the worker's own ledger view, count them free at
    once, so an attach that needs them is refused at admission (UnexpectedAdmissionError; with
    direct binding OutOfamd.com/gpu). The worker retries such a refusal with backoff while its
    view has room, instead of answering a full node's 'Insufficient GPU'."""
    async def main():
        lat = LatencyModel(teardown_ms=150.0)
        async with LocalCluster(latency=lat, worker_overrides=binding) as lc:
            lc.tenant("a")
            lc.tenant("b")
            code, b = await lc.add("default", "a", 8)
            assert code == 200
            code, _ = await lc.remove("default", "a", [d["uuid"] for d in b["devices"]])
            assert code == 200
            code, b = await lc.add("default", "b", 8)
            assert code == 200 and len(b["devices"]) == 8, b
            assert not await lc.audit("default", "b")
            # a node that is really full is still refused at once
            t0 = time.perf_counter()
            code, _ = await lc.add("default", "a", 1)
            assert code == 500 and time.perf_counter() - t0 < 0.5
    asyncio.run(main())


@pytest.mark.parametrize("binding", [{}, DIRECT], ids=["scheduler", "direct"])
def test_the_pool_refills_after_the_kubelet_refused_it_during_a_teardown(binding):
    """Another workload holds every other GPU, and an operator deletes the standby: the refill
    that the delete triggers finds the kubelet still counting the standby's GPU (its teardown
    takes 150 ms here, and a real kubelet's checkpoint keeps a deleted Pod's entry until its
    next Allocate) and no event follows the teardown. The pool counts only Pods the apiserver
    still has, and a kubelet refusal is looked at again shortly: it refills without waiting
    for the next capacity event."""
    async def main():
        lat = LatencyModel(teardown_ms=150.0)
        async with LocalCluster(latency=lat,
                                worker_overrides={**binding, "warm_pool_size": 1}) as lc:
            pool = lc.nodes["node-0"].worker.pool
            end = time.monotonic() + 5
            while len(pool.standby()) < 1:
                assert time.monotonic() < end, "pool not filled at start"
                await asyncio.sleep(0.02)
            sb = pool.standby()[0]
            lc.tenant("hog", gpus=7)                     # every other GPU
            lc.cluster.delete(sb.namespace, sb.name, grace=0)   # an operator deletes the standby
            end = time.monotonic() + 3
            while not [p for p in pool.standby() if p.uid != sb.uid]:
                assert time.monotonic() < end, "pool not refilled after the teardown"
                await asyncio.sleep(0.02)
    asyncio.run(main())


def test_the_pool_refills_although_the_kubelets_checkpoint_still_lists_a_deleted_pod():
    """A real device manager drops a deleted Pod from its books, and from the checkpoint file,
    only at the next Allocate. A pool that counted the checkpoint's entries as allocated would
    see no free GPU after another workload left a full node, create no standby, and so never
    trigger that Allocate. The pool counts only Pods the apiserver still has."""
    async def main():
        async with LocalCluster(lazy_checkpoint=True,
                                worker_overrides={"warm_pool_size": 1}) as lc:
            pool = lc.nodes["node-0"].worker.pool
            end = time.monotonic() + 5
            while len(pool.standby()) < 1:
                assert time.monotonic() < end, "pool not filled at start"
                await asyncio.sleep(0.02)
            sb = pool.standby()[0]
            lc.tenant("hog", gpus=7)
            lc.cluster.delete(sb.namespace, sb.name, grace=0)
            end = time.monotonic() + 3
            while not [p for p in pool.standby() if p.uid != sb.uid]:
                assert time.monotonic() < end, "pool not refilled"
                await asyncio.sleep(0.02)
    asyncio.run(main())
