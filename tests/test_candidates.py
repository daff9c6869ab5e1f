"""A pick's candidate mark seen in a stale cache (worker/reconciler.py follow-up and sweep,
cluster/placeholder.py ``_delete(candidate_only=True)``)."""
import asyncio
import copy

from gpumounter_amd.cluster.pool import is_standby
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.models.types import ANN_CANDIDATE


def test_a_stale_candidate_mark_never_releases_a_mounted_placeholder():
    """Chaos sweep4 f644: a pick's confirm PATCH landed while the placeholder watch relisted;
    the relisted cache still showed the candidate mark, and the attach's follow-up (its
    surplus release had failed) took the mark for a failed pick's and deleted a mounted
    placeholder — the GPU was revoked from the Pod after a 200. The follow-up and the sweep
    now delete a candidate only while the apiserver still shows it one."""
    async def main():
        async with LocalCluster() as lc:
            w = lc.nodes["node-0"].worker
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)
            assert code == 200
            ph = next(p for p in lc.cluster.placeholders() if not is_standby(p))
            key = (ph["metadata"]["namespace"], ph["metadata"]["name"])
            stale = copy.deepcopy(w.service.ph.informer.cache[key])
            stale["metadata"].setdefault("annotations", {})[ANN_CANDIDATE] = "x"
            w.service.ph.informer.cache[key] = stale        # the relisted, pre-confirm view
            w.reconciler.follow_up("default", "t")
            await asyncio.sleep(0.3)
            assert lc.cluster.get(*key) is not None, "mounted placeholder deleted"
            w.service.ph.informer.cache[key] = stale
            await w.reconciler.run_once()
            assert lc.cluster.get(*key) is not None, "mounted placeholder deleted by the sweep"
            assert not await lc.audit("default", "t")
    asyncio.run(main())


def test_a_create_that_failed_after_taking_effect_is_reaped_at_once():
    """Chaos sweep6 pre0660: a placeholder POST took effect but every answer was lost; the
    reservation failed and released what it knew of, and the placeholder it did not know of
    held a GPU until the next periodic sweep (30 s). Its name is the attach's own, so the
    failed reservation reads it back and deletes it at once."""
    async def main():
        async with LocalCluster(worker_overrides={"reconcile_on_events": False}) as lc:
            lc.tenant("t")
            lc.cluster.fail_next("POST", 503, count=20, after=True)
            code, _ = await lc.add("default", "t", 1)
            assert code == 500
            await asyncio.sleep(0.2)
            left = [p["metadata"]["name"] for p in lc.cluster.placeholders()]
            assert not left, f"placeholders left behind: {left}"
            lc.cluster._faults.clear()            # noqa: SLF001 - any left unconsumed
            code, b = await lc.add("default", "t", 8)
            assert code == 200 and len(b["devices"]) == 8
    asyncio.run(main())


def test_a_hold_whose_unschedulable_release_fails_lets_its_admitted_ones_go_too():
    """Chaos sweep9 pre0692: a correction's hold (hold_singles: 1-GPU candidates for every free
    GPU) got some admitted and some unschedulable; releasing the unschedulable ones failed after
    taking effect, the hold raised, and the admitted candidates — which the correction never
    learned of — held their GPUs until the next periodic sweep. Now the hold lets them go too
    (and a correction that gave up hands the Pod to the follow-up)."""
    from gpumounter_amd.utils.faults import FaultInjector, InjectedFault

    async def main():
        async with LocalCluster() as lc:
            ph = lc.nodes["node-0"].worker.service.ph
            owner = lc.tenant("t")
            ph.faults = FaultInjector("ledger_release:1:after")
            try:
                await ph.hold_singles(owner, 10, False, "", "add-x")    # 8 GPUs: 2 refused
            except InjectedFault:
                pass
            else:
                raise AssertionError("the injected release fault did not fire")
            finally:
                ph.faults = FaultInjector("")
            await asyncio.sleep(0.1)
            left = [p["metadata"]["name"] for p in lc.cluster.placeholders()]
            assert not left, f"admitted candidates left behind: {left}"
    asyncio.run(main())


def test_an_attach_into_a_pod_deleted_before_its_placeholders_existed_is_undone():
    """Chaos (box sweep 3, td702): the tenant was deleted and re-created under its name while
    an attach ran, before the attach had created its placeholders. The DELETED event's release
    found nothing to release, the kubelet had not stopped the old containers yet (its teardown
    lags the DELETE), so the mount succeeded and the attach answered 200 — and the placeholders
    of a Pod that no longer existed held their GPUs until the periodic sweep. The attach now
    checks its Pod at the end, releases what it booked and answers PodNotFound."""
    from gpumounter_amd.fakes.apiserver import LatencyModel

    async def main():
        async with LocalCluster(latency=LatencyModel(teardown_ms=500.0),
                                worker_overrides={"reconcile_on_events": True}) as lc:
            svc = lc.nodes["node-0"].worker.service
            old = lc.tenant("t")
            orig = svc.ph.reserve

            async def reserve(*a, **kw):
                svc.ph.reserve = orig
                lc.cluster.delete("default", "t", grace=0)
                lc.tenant("t")                              # the same name, a new UID
                await asyncio.sleep(0.1)                    # the worker's watch sees both
                return await orig(*a, **kw)
            svc.ph.reserve = reserve
            code, body = await lc.add("default", "t", 2)
            assert code != 200, body
            await asyncio.sleep(0.2)
            mine = [p["metadata"]["name"] for p in lc.cluster.placeholders()
                    if (p["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/owner-uid") == old["metadata"]["uid"]]
            assert not mine, f"placeholders of the deleted Pod left: {mine}"
    asyncio.run(main())
