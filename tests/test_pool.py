"""Warm placeholder pool (gpumounter_amd/cluster/pool.py): claims skip scheduling + admission,
detaches hand GPUs back, entire mounts keep all-or-nothing semantics, the ledger stays consistent."""
import asyncio
import time

import pytest

from gpumounter_amd.cluster.pool import is_standby
from gpumounter_amd.fakes.apiserver import LatencyModel
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.models.device import normalize_device_id


async def wait_pool(lc, n, timeout=5.0):
    pool = lc.nodes["node-0"].worker.pool
    t0 = time.monotonic()
    while len(pool.standby()) < n:
        assert time.monotonic() - t0 < timeout, (len(pool.standby()), n)
        await asyncio.sleep(0.01)
    return pool


def standby_count(lc):
    return sum(1 for p in lc.cluster.placeholders() if is_standby(p))


def test_pool_fills_claims_and_takes_back():
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 8}) as lc:
            await wait_pool(lc, 8)
            assert len(lc.nodes["node-0"].node.allocated) == 8      # held in the books
            lc.tenant("t")
            posts = lc.cluster.requests_by_verb.get("POST", 0)
            code, b = await lc.add("default", "t", 2)
            assert code == 200
            assert lc.cluster.requests_by_verb.get("POST", 0) == posts  # no placeholder created
            assert {t["name"] for t in b["timings"]} >= {"pool_claim"}
            assert [d["numa_node"] for d in b["devices"]] == [0, 0]
            assert not await lc.audit("default", "t")
            assert standby_count(lc) == 6 and len(lc.cluster.placeholders()) == 8
            code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
            assert code == 200 and not await lc.audit("default", "t")
            await wait_pool(lc, 8)
            assert standby_count(lc) == 8 and len(lc.nodes["node-0"].node.allocated) == 8
    asyncio.run(main())


def test_pool_entire_mount_group_semantics():
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 8}) as lc:
            await wait_pool(lc, 8)
            lc.tenant("e")
            code, b = await lc.add("default", "e", 4, entire=True)
            assert code == 200 and len(b["devices"]) == 4
            assert (await lc.add("default", "e", 1))[0] == 500          # entire: no more adds
            ids = [d["uuid"] for d in b["devices"]]
            assert (await lc.remove("default", "e", ids[:2]))[0] == 400  # whole group only
            assert (await lc.remove("default", "e", ids))[0] == 200
            assert not await lc.audit("default", "e")
    asyncio.run(main())


def test_pool_partial_cover_mixes_claim_and_create():
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 2}) as lc:
            await wait_pool(lc, 2)
            lc.tenant("m")
            code, b = await lc.add("default", "m", 5)
            assert code == 200 and len(b["devices"]) == 5
            assert not await lc.audit("default", "m")
            node = lc.nodes["node-0"].node
            # 5 hot + refilled standby ≤ 8, never double-booked
            assert len(node.allocated) <= 8 and len(set(node.allocated)) == len(node.allocated)
            code, _ = await lc.remove("default", "m", [d["uuid"] for d in b["devices"]])
            assert code == 200 and not await lc.audit("default", "m")
            await wait_pool(lc, 2)
    asyncio.run(main())


def test_pool_takes_scheduling_and_admission_off_the_attach_path():
    """Counted in control-plane phases, not wall-clock ratios (a ratio of medians flaked under
    a loaded ``-n 8`` run): a cold attach creates a placeholder and waits for the scheduler and
    the kubelet (≥ schedule_ms + admit_ms of the fake's latency model); a warm one claims a
    standby placeholder with a metadata patch and waits for neither."""
    lat = LatencyModel(api_ms=0.5, schedule_ms=10, admit_ms=15, sandbox_ms=50, start_ms=20)

    async def measure(pool_size):
        async with LocalCluster(latency=lat, worker_overrides={"warm_pool_size": pool_size}) as lc:
            if pool_size:
                await wait_pool(lc, pool_size, timeout=10)
            lc.tenant("x")
            out = []
            for _ in range(5):
                t0 = time.perf_counter()
                code, b = await lc.add("default", "x", 1)
                ms = (time.perf_counter() - t0) * 1e3
                assert code == 200
                out.append((ms, {t["name"] for t in b.get("timings", [])}))
                await lc.remove("default", "x", [b["devices"][0]["uuid"]])
                if pool_size:
                    await wait_pool(lc, pool_size, timeout=10)
            return out

    async def main():
        for ms, stages in await measure(0):
            assert ms > 25                                  # schedule + admission are waited on
            assert any(s.endswith("placeholder_wait") for s in stages), stages
            assert not any(s.endswith("pool_claim") for s in stages), stages
        for ms, stages in await measure(4):
            assert any(s.endswith("pool_claim") for s in stages), stages
            assert not any(s.endswith("placeholder_wait") or s.endswith("ledger_reserve")
                           for s in stages), stages
    asyncio.run(main())


def test_attach_during_a_refill_claims_the_new_standby_gpus():
    """A refill that started before an attach holds the node's last free GPUs in standby
    placeholders that are bound but not admitted yet. The attach's plan sees those GPUs as
    free and its creates are unschedulable: it then waits for the refill's admission and
    claims the new standby GPUs instead of answering "insufficient" with GPUs to spare
    (found by the ledger state machine, tests/test_ledger_model.py)."""
    lat = LatencyModel(schedule_ms=2, admit_ms=400)

    async def main():
        async with LocalCluster(latency=lat, worker_overrides={"warm_pool_size": 2}) as lc:
            pool = await wait_pool(lc, 2, timeout=10)
            lc.tenant("a")
            lc.tenant("b")
            code, b = await lc.add("default", "a", 5)          # 2 claimed + 3 created: 3 free
            assert code == 200
            t0 = time.monotonic()
            while not pool.refilling():
                assert time.monotonic() - t0 < 5, "the refill never started"
                await asyncio.sleep(0.002)
            assert not pool.standby()                           # bound, not admitted yet
            code, b = await lc.add("default", "b", 2)
            assert code == 200, b
            assert {t["name"] for t in b["timings"]} >= {"pool_claim"}
            assert not await lc.audit("default", "b") and not await lc.audit("default", "a")
    asyncio.run(main())


def test_pool_claims_released_when_tenant_disappears():
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 4}) as lc:
            await wait_pool(lc, 4)
            lc.tenant("gone")
            code, b = await lc.add("default", "gone", 2)
            assert code == 200
            lc.cluster.delete("default", "gone", grace=0)
            # the worker reacts to the tenant's DELETED event at once; the reconciler's sweep
            # collects whatever that left (which of the two gets a placeholder is a race)
            rep = await lc.nodes["node-0"].worker.reconciler.run_once()
            assert len(rep.owner_gone) <= 2

            def owned_by_gone():
                return [p for p in lc.cluster.placeholders() if (p["metadata"].get(
                    "annotations") or {}).get("gpumounter.amd.com/owner-name") == "gone"]
            for _ in range(200):
                if not owned_by_gone():
                    break
                await asyncio.sleep(0.01)
            assert owned_by_gone() == []
            await wait_pool(lc, 4)
            assert standby_count(lc) == 4
    asyncio.run(main())


def test_failed_claim_whose_patch_took_effect_is_undone():
    """A claim PATCH that the apiserver applied but whose reply never arrived (every retry's too)
    looks failed. The attach falls back to other GPUs, so that placeholder must not stay the
    tenant's: it is put back into the pool (or deleted), never left as a GPU the tenant was told
    it did not get."""
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 2}) as lc:
            await wait_pool(lc, 2)
            lc.tenant("t")
            # both claim PATCHes, first attempt and every retry (5 each): applied, reply lost
            lc.cluster.fail_next("PATCH", 503, count=10, after=True)
            code, b = await lc.add("default", "t", 2)
            assert code == 200
            got = {d["uuid"] for d in b["devices"]}
            svc = lc.nodes["node-0"].worker.service
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            assert {g.uuid for g in st.hot} == got          # nothing beyond what was answered
            owned = [p for p in lc.cluster.placeholders()
                     if (p["metadata"].get("annotations") or {}).get(
                         "gpumounter.amd.com/owner-name") == "t"]
            assert sum(int(c["resources"]["limits"]["amd.com/gpu"])
                       for p in owned for c in p["spec"]["containers"]) == 2
            assert not await lc.audit("default", "t")
    asyncio.run(main())


def owner_of(lc, name):
    return (lc.cluster.get("gpu-pool", name)["metadata"].get("annotations") or {}).get(
        "gpumounter.amd.com/owner-name")


def test_claim_of_a_placeholder_taken_meanwhile_never_double_books():
    """The worker's cache can be behind the apiserver: after a relist an acknowledged claim is
    not in it yet, and a worker SIGKILLed mid-claim can still have a PATCH in flight. A claim
    planned on that cache must not overwrite the other claim (bench/configs.py chaos, warm pool
    2, seed 90: two Pods answered 200 for the same two GPUs). The claim is conditional on the
    version it was planned on, so it fails, and the one it lost to keeps the placeholder."""
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 1}) as lc:
            pool = await wait_pool(lc, 1)
            lc.tenant("a")
            lc.tenant("b")
            (ph,) = pool.standby()
            # b's claim lands at the apiserver; nothing has yielded to the informer since
            b = lc.cluster.get("default", "b")
            lc.cluster.patch("gpu-pool", ph.name, {"metadata": {"annotations": {
                "gpumounter.amd.com/owner-name": "b",
                "gpumounter.amd.com/owner-uid": b["metadata"]["uid"],
                "gpumounter.amd.com/mount-mode": "single",
                "gpumounter.amd.com/attach-id": "add-b"}}})
            a = lc.cluster.get("default", "a")
            got = await pool.claim(a, 1, False, [], attach_id="add-a")
            assert got is None                      # the caller falls back to creating
            assert owner_of(lc, ph.name) == "b"     # b's claim stands
    asyncio.run(main())


@pytest.mark.parametrize("room", [False, True], ids=["pool-full-delete", "pool-room-patch"])
def test_give_back_leaves_a_placeholder_claimed_anew_with_its_new_owner(room):
    """A give-back planned on a stale cache (the placeholder already went back to the pool and
    was claimed by another Pod) must not take it from that Pod: neither put it back into the
    pool (room in the pool) nor delete it (pool full)."""
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 1}) as lc:
            pool = await wait_pool(lc, 1)
            svc = lc.nodes["node-0"].worker.service
            lc.tenant("a")
            lc.tenant("b")
            code, _ = await lc.add("default", "a", 1)
            assert code == 200
            (p,) = svc.ph.owned_by(lc.cluster.get("default", "a"))
            ph = svc.ph.cached(p)
            b = lc.cluster.get("default", "b")
            lc.cluster.patch("gpu-pool", ph.name, {"metadata": {"annotations": {
                "gpumounter.amd.com/owner-name": "b",
                "gpumounter.amd.com/owner-uid": b["metadata"]["uid"],
                "gpumounter.amd.com/attach-id": "add-b"}}})
            if room:
                pool.target = 3
            await pool.give_back([ph])
            assert owner_of(lc, ph.name) == "b"
    asyncio.run(main())


@pytest.mark.parametrize("room", [True, False])
def test_a_late_follow_up_leaves_a_slave_pod_claimed_from_the_pool_with_its_holder(room):
    """A failed attach hands its placeholders to the reconciler's follow-up. One of them, a
    ``<pod>-slave-pod-`` (not a ``gpumounter-standby-`` name: a pick's surplus goes back to the
    pool under its own name), went back to the pool and another Pod claimed it. The follow-up
    must neither return it to the pool nor delete it, and the failed attach's 'abandoned' mark
    must not hide it from its new owner's ledger view (chaos seed 114 saw a slave pod claimed
    from the pool; the delete path only checked holders of ``gpumounter-standby-`` names)."""
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 1,
                                                  "reconcile_on_events": False}) as lc:
            pool = await wait_pool(lc, 1)
            w = lc.nodes["node-0"].worker
            svc = w.service
            lc.tenant("a")
            lc.tenant("b")
            a, b = lc.cluster.get("default", "a"), lc.cluster.get("default", "b")
            res = await svc.ph.reserve(a, 1, False, attach_id="add-a")
            (ph,) = res.placeholders
            assert ph.name.startswith("a-slave-pod-") and ph.owner_uid == a["metadata"]["uid"]
            assert await pool._put_back(ph, ph.held_by_me) is True       # back in the pool
            idx = lc.inventory.by_key()[normalize_device_id(ph.device_ids[0])].index
            got = await pool.claim(b, 1, False, [], attach_id="add-b", want=[idx])
            assert got is not None and got.placeholders[0].name == ph.name
            if not room:
                pool.target = 0
            svc._follow_up(a, [ph])            # the failed attach's follow-up, late
            for _ in range(100):
                await asyncio.sleep(0.01)
                if not svc.abandoned:
                    break
            assert owner_of(lc, ph.name) == "b"
            st = await svc.pod_state(lc.cluster.get("default", "b"), fresh=True)
            assert [p.name for p in st.placeholders] == [ph.name]
    asyncio.run(main())


def test_release_of_a_placeholder_in_status_churn_still_deletes_it():
    """Releases are conditional on the placeholder's version. One being admitted changes with
    every status the kubelet posts, so a release right after its create meets conflicts with
    the holder unchanged: it must retry through them, not give up after three and leave the
    GPU booked under an attach that failed (chaos seeds 120, 121, 123)."""
    async def main():
        async with LocalCluster() as lc:
            svc = lc.nodes["node-0"].worker.service
            lc.tenant("a")
            res = await svc.ph.reserve(lc.cluster.get("default", "a"), 1, False,
                                       attach_id="add-a")
            (ph,) = res.placeholders
            delete, churn = svc.ph.kube.delete_pod, [5]

            async def churning(ns, name, **kw):
                if churn[0]:                   # a status update lands first, five times
                    churn[0] -= 1
                    lc.cluster.patch(ns, name, {"metadata": {"annotations": {
                        "churn": str(churn[0])}}})
                return await delete(ns, name, **kw)
            svc.ph.kube.delete_pod = churning
            await svc.ph.release([ph])
            assert lc.cluster.get(ph.namespace, ph.name) is None
    asyncio.run(main())


def test_claim_whose_reply_was_lost_is_kept():
    """A conditional claim whose first attempt applied but whose reply was lost meets a
    conflict on its retry; the placeholder read back is this attach's own, so the claim
    stands (no fallback, no placeholder created)."""
    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 2}) as lc:
            await wait_pool(lc, 2)
            lc.tenant("t")
            lc.cluster.fail_next("PATCH", 503, count=1, after=True)
            code, b = await lc.add("default", "t", 1)
            assert code == 200
            stages = {t["name"] for t in b["timings"]}
            assert "pool_claim" in stages and not any(
                s.endswith("placeholder_wait") for s in stages), stages
            assert owner_of(lc, b["devices"][0]["placeholder"]) == "t"
            assert not await lc.audit("default", "t")
    asyncio.run(main())


def test_pick_surplus_returned_to_the_pool_is_no_candidate_for_its_next_owner():
    """A trim/correction pick holds every free GPU with *candidate* placeholders and gives the
    surplus back to the warm pool. Back in the pool they must lose the candidate mark: a
    tenant that later claimed one would otherwise not see it in its ledger view (candidates are
    nobody's yet), the audit would call its mounted GPU stale, and the reconciler would release
    it as an abandoned pick — the GPU back to the scheduler, the tenant still using it."""
    from gpumounter_amd.models.types import ANN_CANDIDATE

    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 1}) as lc:
            pool = await wait_pool(lc, 1)
            w = lc.nodes["node-0"].worker
            svc = w.service
            lc.tenant("a")
            lc.tenant("b")
            a = lc.cluster.get("default", "a")
            held = await svc.ph.hold_singles(a, 2, False, "", "rid-pick", "", "")
            assert len(held) == 2 and all(p.candidate for p in held)
            pool.target = 3                      # room for both
            await pool.give_back(held)
            back = [p for p in lc.cluster.placeholders()
                    if p["metadata"]["name"] in {h.name for h in held}]
            assert len(back) == 2 and all(is_standby(p) for p in back)
            assert not any(ANN_CANDIDATE in (p["metadata"].get("annotations") or {})
                           for p in back)
            pool.target = 1
            code, b = await lc.add("default", "b", 3)
            assert code == 200
            owned = svc.ph.owned_by(lc.cluster.get("default", "b"))
            assert sum(len(svc.ph.cached(p).device_ids) for p in owned) == 3
            assert not await lc.audit("default", "b")
            await w.reconciler.run_once()
            assert len(svc.ph.owned_by(lc.cluster.get("default", "b"))) == len(owned)
            assert not await lc.audit("default", "b")
    asyncio.run(main())


def test_release_of_a_claimed_placeholder_behind_a_stale_cache_still_deletes_it():
    """The worker's cache can still show a placeholder as standby after this worker claimed it
    (the claim's write-through was dropped by a relist). Releasing it for its owner must still
    delete it: the owner that counts is the one the releasing caller's view holds, not the
    stale cache's."""
    import copy

    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 1}) as lc:
            pool = await wait_pool(lc, 1)
            svc = lc.nodes["node-0"].worker.service
            lc.tenant("a")
            (ph,) = pool.standby()
            key = (ph.namespace, ph.name)
            stale = copy.deepcopy(svc.ph.informer.cache[key])
            got = await pool.claim(lc.cluster.get("default", "a"), 1, False, [],
                                   attach_id="add-a")
            assert got is not None and got.placeholders[0].owner_uid
            svc.ph.informer.cache[key] = stale          # the claim never reached the cache
            await svc.ph.release(got.placeholders)
            assert lc.cluster.get(*key) is None
    asyncio.run(main())


def test_a_claim_overtaken_by_a_relist_is_not_revoked_by_the_reconciler():
    """A relist between a claim PATCH and its reply drops the claim's write-through: until a GET
    settles the key the cache shows the placeholder standby. A reconcile of the owner in that
    window saw its just-mounted GPU as stale and revoked it, and nothing repaired it until the
    next sweep (chaos: trim + warm pool + leases, seed 72). reconcile_pod now waits for the view
    to settle."""
    import copy

    async def main():
        async with LocalCluster(worker_overrides={"warm_pool_size": 1}) as lc:
            pool = await wait_pool(lc, 1)
            svc = lc.nodes["node-0"].worker.service
            inf = svc.ph.informer
            lc.tenant("a")
            (ph,) = pool.standby()
            key = (ph.namespace, ph.name)
            before = copy.deepcopy(inf.cache[key])
            real_patch, real_fetch = svc.ph.kube.patch_pod, inf._fetch     # noqa: SLF001

            async def patch(ns, name, body):
                out = await real_patch(ns, name, body)
                if name == ph.name and (body["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/owner-name") == "a":
                    inf.epoch += 1                   # a relist listed the pre-claim version
                    inf.cache[key] = copy.deepcopy(before)
                return out

            async def slow_fetch(k):
                if k == key:
                    await asyncio.sleep(0.3)
                return await real_fetch(k)
            svc.ph.kube.patch_pod, inf._fetch = patch, slow_fetch               # noqa: SLF001
            inf._task.cancel()          # the resumed watch has not delivered the claim yet
            await asyncio.sleep(0)
            code, b = await lc.add("default", "a", 1)
            assert code == 200 and b["devices"][0]["placeholder"] == ph.name
            assert not getattr(inf, "settled", False)      # the GET is still on its way
            await svc.reconcile_pod(lc.cluster.get("default", "a"))
            await asyncio.sleep(0.5)                 # the GET has settled the view
            assert inf.cache[key]["metadata"]["annotations"].get(
                "gpumounter.amd.com/owner-name") == "a"
            assert not await lc.audit("default", "a")   # still mounted: nothing was revoked
    asyncio.run(main())


def test_a_second_attach_behind_an_overtaken_claim_keeps_the_first_gpu():
    """The same window for the attach path: a Pod's next attach computes the complete set of
    nodes its container keeps (cgroup v2 writes the whole allow set) from the Pod's view. Taken
    before the relist-overtaken claim settles, that set left the first GPU out and its access was
    revoked by the second attach."""
    import copy

    async def main():
        async with LocalCluster(cgroup_mode="v2", worker_overrides={"warm_pool_size": 1}) as lc:
            pool = await wait_pool(lc, 1)
            svc = lc.nodes["node-0"].worker.service
            inf = svc.ph.informer
            lc.tenant("a")
            (ph,) = pool.standby()
            key = (ph.namespace, ph.name)
            before = copy.deepcopy(inf.cache[key])
            real_patch, real_fetch = svc.ph.kube.patch_pod, inf._fetch     # noqa: SLF001

            async def patch(ns, name, body):
                out = await real_patch(ns, name, body)
                if name == ph.name and (body["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/owner-name") == "a":
                    inf.epoch += 1
                    inf.cache[key] = copy.deepcopy(before)
                return out

            async def slow_fetch(k):
                if k == key:
                    await asyncio.sleep(0.3)
                return await real_fetch(k)
            svc.ph.kube.patch_pod, inf._fetch = patch, slow_fetch               # noqa: SLF001
            inf._task.cancel()
            await asyncio.sleep(0)
            code, first = await lc.add("default", "a", 1)
            assert code == 200 and first["devices"][0]["placeholder"] == ph.name
            code, second = await lc.add("default", "a", 1)
            assert code == 200
            await asyncio.sleep(0.5)
            assert not await lc.audit("default", "a")
    asyncio.run(main())
