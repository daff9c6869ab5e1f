"""GPU leases (gpumounter_amd/worker/lease.py): ``?lease=<s>`` attaches that detach themselves."""
import asyncio
import subprocess
import time

import pytest

from gpumounter_amd import _native
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.worker.lease import ANN_LEASE


def run(coro_fn, **kw):
    async def main():
        async with LocalCluster(**kw) as lc:
            return await coro_fn(lc)
    return asyncio.run(main())


async def lease_add(lc, ns, pod, n, lease, entire=False):
    url = (f"{lc.master_url}/addgpu/namespace/{ns}/pod/{pod}/gpu/{n}/isEntireMount/"
           f"{'true' if entire else 'false'}?lease={lease}")
    async with lc.session.get(url, headers={"Accept": "application/json"}) as r:
        return r.status, await r.json()


async def until(pred, timeout=5.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if await pred():
            return True
        await asyncio.sleep(0.02)
    return await pred()


def test_lease_detaches_on_time_and_only_the_leased_gpus():
    async def body(lc):
        lc.tenant("t")
        code, keep = await lc.add("default", "t", 1)                  # no lease
        assert code == 200
        code, b = await lease_add(lc, "default", "t", 2, 0.3)
        assert code == 200 and "(lease until " in b["detail"], b
        leased = {p["metadata"]["name"] for p in lc.cluster.placeholders()
                  if (p["metadata"].get("annotations") or {}).get(ANN_LEASE)}
        assert len(leased) == 2
        svc = lc.nodes["node-0"].worker.service

        async def back_to_one():
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            return [g.uuid for g in st.hot] == [keep["devices"][0]["uuid"]]
        assert await until(back_to_one)
        assert await lc.audit("default", "t") == []

        async def expired_events():   # emitted once remove_gpu has returned to the lease
            await svc.notify.drain()
            return [e for e in lc.cluster.events_for("default", "t")
                    if e["reason"] == "GPULeaseExpired"]
        assert await until(expired_events)
        evs = await expired_events()
        assert evs and "2 GPU(s) detached" in evs[0]["message"] and evs[0]["type"] == "Normal"
        assert svc.lease.expired == 1
    run(body)


def test_bad_lease_values_are_rejected():
    async def body(lc):
        lc.tenant("t")
        for v in ("-1", "0", "abc", "inf"):
            code, b = await lease_add(lc, "default", "t", 1, v)
            assert code == 400 and "Invalid param lease" in b["message"], (v, b)
    run(body)


def test_expired_lease_on_a_busy_gpu_is_kept_unless_forced(tmp_path):
    sleeper = subprocess.Popen(["sleep", "60"])
    procs = tmp_path / "procs"
    try:
        async def body(lc):
            # after the cluster's inventory ran amdsmi_init, which resets the mock's settings
            _native.mock_smi().gm_mock_set_procs_file(str(procs).encode())
            lc.tenant("busy", pids={"main": [sleeper.pid]})
            code, b = await lease_add(lc, "default", "busy", 1, 1.0)   # > procs write under load
            assert code == 200
            procs.write_text(f"{b['devices'][0]['index']} {sleeper.pid} 4096 python\n")
            svc = lc.nodes["node-0"].worker.service

            async def warned():
                await svc.notify.drain()
                return any(e["reason"] == "GPULeaseExpired" and e["type"] == "Warning"
                           for e in lc.cluster.events_for("default", "busy"))
            assert await until(warned)
            st = await svc.pod_state(lc.cluster.get("default", "busy"), fresh=True)
            assert len(st.hot) == 1                       # still mounted: a process uses it
            svc.cfg.lease_force = True                    # operator flips the policy
            svc.lease._retry_after.clear()                # noqa: SLF001 - retry now
            await svc.lease.sweep()

            async def gone():
                st = await svc.pod_state(lc.cluster.get("default", "busy"), fresh=True)
                return not st.hot
            assert await until(gone)
            assert await lc.audit("default", "busy") == []
        run(body, worker_overrides={"busy_detection": "both", "lease_retry_s": 0.1})
        sleeper.wait(timeout=10)
        assert sleeper.returncode == -15                  # SIGTERM like force=1
    finally:
        _native.mock_smi().gm_mock_set_procs_file(b"")
        if sleeper.poll() is None:
            sleeper.kill()


def test_a_busy_expired_lease_does_not_hold_back_the_owners_next_lease(tmp_path):
    """An expired lease whose GPU is busy is retried every lease_retry_s. That retry gate is
    the busy placeholder's: a second lease of the same Pod on another GPU still ends on time
    (it used to wait for the whole retry period, found by chaos with the warm pool and leases:
    a concurrent RemoveGPU made an expiry answer GPU_NOT_FOUND and gated the owner)."""
    sleeper = subprocess.Popen(["sleep", "60"])
    procs = tmp_path / "procs"
    try:
        async def body(lc):
            _native.mock_smi().gm_mock_set_procs_file(str(procs).encode())
            lc.tenant("busy", pids={"main": [sleeper.pid]})
            code, b = await lease_add(lc, "default", "busy", 1, 1.0)
            assert code == 200
            procs.write_text(f"{b['devices'][0]['index']} {sleeper.pid} 4096 python\n")
            svc = lc.nodes["node-0"].worker.service

            async def warned():
                await svc.notify.drain()
                return any(e["reason"] == "GPULeaseExpired" and e["type"] == "Warning"
                           for e in lc.cluster.events_for("default", "busy"))
            assert await until(warned)
            code, c = await lease_add(lc, "default", "busy", 1, 0.3)
            assert code == 200
            second = c["devices"][0]["uuid"]

            async def second_gone():
                st = await svc.pod_state(lc.cluster.get("default", "busy"), fresh=True)
                return second not in {g.uuid for g in st.hot} and len(st.hot) == 1
            assert await until(second_gone, timeout=3.0)
        run(body, worker_overrides={"busy_detection": "both", "lease_retry_s": 30.0})
    finally:
        _native.mock_smi().gm_mock_set_procs_file(b"")
        sleeper.kill()
        sleeper.wait(timeout=10)


def test_lease_survives_a_worker_restart():
    async def body(lc):
        lc.tenant("t")
        code, _ = await lease_add(lc, "default", "t", 1, 0.4)
        assert code == 200
        await lc.stop_worker("node-0")                   # timers die with the process
        await asyncio.sleep(0.6)                         # the lease expires meanwhile
        await lc.start_worker("node-0")                  # start-up sweep finds it
        svc = lc.nodes["node-0"].worker.service

        async def gone():
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            return not st.hot
        assert await until(gone)
        assert await lc.audit("default", "t") == []
    run(body)


def test_stop_cancels_timers_and_lets_a_running_expiry_finish():
    """Worker shutdown: armed lease timers never fire afterwards, and an expiry that is already
    detaching finishes (within the grace) instead of running on against closed clients."""
    from gpumounter_amd.worker.lease import LeaseKeeper

    calls = []

    class Svc:
        pass

    async def main():
        lk = LeaseKeeper(Svc())

        async def slow_expire(ns, name):
            calls.append(("start", name))
            await asyncio.sleep(0.05)
            calls.append(("done", name))
        lk.expire_owner = slow_expire
        import time as _t
        lk._arm("u1", "ns", "now", _t.time())          # noqa: SLF001 - fires at once
        lk._arm("u2", "ns", "later", _t.time() + 0.2)  # noqa: SLF001
        await asyncio.sleep(0.01)                        # "now" is mid-expiry
        await lk.stop()
        await asyncio.sleep(0.3)                         # "later" would have fired by now
        lk._arm("u3", "ns", "after-stop", _t.time())   # noqa: SLF001 - ignored once stopped
        await asyncio.sleep(0.02)
    asyncio.run(main())
    assert calls == [("start", "now"), ("done", "now")]


def test_a_retried_leased_attach_cut_off_before_its_lease_still_expires():
    """The worker is killed after mounting a leased attach but before the lease annotation is
    written; the master retries AddGPU under the same idempotency key on the next worker, which
    replays the attach. The replay must record the lease, or the GPUs it hands back as leased
    never expire (chaos --lease-rate: a lease lost across a worker SIGKILL)."""
    from gpumounter_amd.api import gpu_mount as api

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        # the cut-off first attempt: mounted under key K, no lease recorded
        resp = await svc.add_gpu(api.AddGPURequest(pod_name="t", namespace="default", gpu_num=1,
                                                   idempotency_key="K", lease_s=0))
        assert resp.add_gpu_result == api.ADD_SUCCESS
        url = f"{lc.master_url}/addgpu/namespace/default/pod/t/gpu/1/isEntireMount/false?lease=0.3"
        async with lc.session.get(url, headers={"Accept": "application/json",
                                                "Idempotency-Key": "K"}) as r:
            code, b = r.status, await r.json()
        assert code == 200 and "(replayed)" in b["detail"], b
        assert [d["uuid"] for d in b["devices"]] == [resp.devices[0].uuid]

        async def gone():
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            return not st.hot
        assert await until(gone, timeout=3.0), "the replayed lease never expired"
        assert await lc.audit("default", "t") == []
    run(body)                  # LocalCluster runs no periodic sweep


def test_a_lease_whose_watch_echo_lags_still_expires():
    """The placeholder informer has not seen the lease annotation (the watch echo of the PATCH
    is late: a dropped stream, a relist) when the lease timer fires. The expiry must not be
    lost: the timer found nothing due, and nothing re-armed it until the periodic sweep."""
    import copy

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        code, b = await lease_add(lc, "default", "t", 1, 0.3)
        assert code == 200, b
        inf = svc.ph.informer
        (key,) = [k for k, p in inf.cache.items()
                  if (p["metadata"].get("annotations") or {}).get(ANN_LEASE)]
        real = inf.cache[key]
        stale = copy.deepcopy(real)
        del stale["metadata"]["annotations"][ANN_LEASE]
        inf.cache[key] = stale                       # the cache as of before our PATCH
        await asyncio.sleep(0.6)                     # the lease timer fires meanwhile
        if inf.cache.get(key) is stale:
            inf.cache[key] = real                    # the late watch event

        async def gone():
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            return not st.hot
        assert await until(gone, timeout=3.0), "the lease was lost"
    run(body)                  # LocalCluster runs no periodic sweep


def test_a_leased_placeholder_admitted_after_its_lease_timer_fired_still_expires():
    """A leased attach's placeholder was still Pending (no GPU free: a dead worker's attach, a
    scheduler slower than the lease) when its lease timer fired: the expiry found nothing to
    detach. The scheduler admits it later and the reconciler mounts it; its lease is long over,
    and nothing but the next periodic sweep (30 s) would expire it (chaos tpr241: a GPU held
    2.6 s past its lease, until the next worker restart)."""
    async def body(lc):
        lc.tenant("hog")
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        code, b = await lc.add("default", "hog", 8)
        assert code == 200, b
        t = lc.cluster.get("default", "t")
        ph = svc.ph.build(t, 1, "single", [], "add-dead-worker", "", "", time.time() + 0.2)
        await svc.kube.create_pod(ph["metadata"]["namespace"], ph)
        await until(lambda: _seen(svc, ph))
        await svc.lease.sweep(expire_due=False)      # a restarted worker re-arms its timer
        await asyncio.sleep(0.5)                     # fired: the placeholder holds no GPU yet
        code, _ = await lc.remove("default", "hog", [d["uuid"] for d in b["devices"]])
        assert code == 200

        async def admitted_and_gone():
            live = [p for p in svc.ph.live()
                    if p["metadata"]["name"] == ph["metadata"]["name"]]
            return not live and not (await svc.pod_state(t, fresh=True)).hot
        assert await until(admitted_and_gone, timeout=3.0), "the late-admitted lease stayed"
        assert await lc.audit("default", "t") == []
    run(body)                  # LocalCluster runs no periodic sweep


async def _seen(svc, ph):
    return any(p["metadata"]["name"] == ph["metadata"]["name"] for p in svc.ph.live())


def test_a_pool_placeholder_does_not_carry_its_last_owners_lease():
    """Warm pool: a leased GPU removed before its expiry goes back to the pool, and the next Pod
    claims that very placeholder. The earlier owner's lease (the annotation, the grant the
    worker remembers) must not expire the new owner's GPU."""
    async def body(lc):
        w = lc.nodes["node-0"].worker
        svc = w.service
        pool = w.pool
        for _ in range(250):
            if len(pool.standby()) == 1:
                break
            await asyncio.sleep(0.02)
        lc.tenant("a")
        lc.tenant("b")
        code, a = await lease_add(lc, "default", "a", 1, 0.4)
        assert code == 200
        ph, idx = a["devices"][0]["placeholder"], a["devices"][0]["index"]
        for _ in range(250):                     # the refill (once the attach is over)
            if len(pool.standby()) == 1 and not pool.pending():
                break
            await asyncio.sleep(0.02)
        pool.target = 2                          # room for it back in the pool
        code, _ = await lc.remove("default", "a", [a["devices"][0]["uuid"]])
        assert code == 200
        got = await pool.claim(lc.cluster.get("default", "b"), 1, False, [],
                               attach_id="add-b", want=[idx])
        assert got is not None and got.placeholders[0].name == ph     # the same placeholder
        await asyncio.sleep(0.6)                 # a's lease would be over by now
        await svc.lease.sweep()
        await asyncio.sleep(0.1)
        owner = (lc.cluster.get("gpu-pool", ph)["metadata"].get("annotations") or {}).get(
            "gpumounter.amd.com/owner-name")
        assert owner == "b" and svc.lease.expired == 0
    run(body, worker_overrides={"warm_pool_size": 1})


def test_the_pod_gpu_view_shows_when_a_lease_ends():
    async def body(lc):
        lc.tenant("t")
        code, plain = await lc.add("default", "t", 1)
        assert code == 200
        code, leased = await lease_add(lc, "default", "t", 1, 60)
        assert code == 200
        url = f"{lc.master_url}/api/v1/namespaces/default/pods/t/gpus"
        async with lc.session.get(url) as r:
            assert r.status == 200
            view = {g["uuid"]: g for g in (await r.json())["gpus"]
                    if g["source"] == "hot-mount"}
        assert view[plain["devices"][0]["uuid"]]["lease_expires"] is None
        exp = view[leased["devices"][0]["uuid"]]["lease_expires"]
        assert exp is not None and 50 < exp - time.time() <= 60
    run(body)


def test_the_pod_gpu_view_leaves_out_placeholders_being_released():
    """A failed attach's leftover that the follow-up is still deleting (chaos v1pl235: a
    placement correction's held GPU whose release failed) and an unconfirmed candidate are not
    the Pod's GPUs: the worker's own ledger view leaves them out, and so must the API's."""
    from gpumounter_amd.models.types import ANN_CANDIDATE

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        code, b = await lc.add("default", "t", 3)
        assert code == 200
        phs = sorted(svc.ph.owned_by(lc.cluster.get("default", "t")),
                     key=lambda p: p["metadata"]["name"])
        assert len(phs) == 3
        left, cand = phs[0], phs[1]
        svc.abandoned[left["metadata"]["uid"]] = (
            left["metadata"]["annotations"]["gpumounter.amd.com/owner-uid"], "")
        key = (cand["metadata"]["namespace"], cand["metadata"]["name"])
        await svc.kube.patch_pod(*key, {"metadata": {"annotations": {ANN_CANDIDATE: "add-x"}}})

        async def marked():
            return ANN_CANDIDATE in svc.ph.informer.cache[key]["metadata"]["annotations"]
        assert await until(marked)
        url = f"{lc.master_url}/api/v1/namespaces/default/pods/t/gpus"
        async with lc.session.get(url) as r:
            assert r.status == 200
            hot = [g for g in (await r.json())["gpus"] if g["source"] == "hot-mount"]
        st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
        assert sorted(g["uuid"] for g in hot) == sorted(g.uuid for g in st.hot)
        assert len(hot) == 1
    run(body)


def test_a_pool_placeholder_reclaimed_by_the_same_pod_does_not_inherit_its_old_lease():
    """The same Pod gives a leased pool placeholder back before the lease ends and a later
    attach of that Pod (no lease) claims the same placeholder: the worker's memory of the old
    grant is for the earlier attach only (found by chaos: warm pool 2, leases, seed 33)."""
    async def body(lc):
        w = lc.nodes["node-0"].worker
        svc, pool = w.service, w.pool
        for _ in range(250):
            if len(pool.standby()) == 1:
                break
            await asyncio.sleep(0.02)
        lc.tenant("a")
        code, a = await lease_add(lc, "default", "a", 1, 0.4)
        assert code == 200
        ph, idx = a["devices"][0]["placeholder"], a["devices"][0]["index"]
        for _ in range(250):        # the refill after the claim is done: room for one give-back
            if len(pool.standby()) == 1 and not pool.refilling():
                break
            await asyncio.sleep(0.02)
        pool.target = 2
        code, _ = await lc.remove("default", "a", [a["devices"][0]["uuid"]])
        assert code == 200
        got = await pool.claim(lc.cluster.get("default", "a"), 1, False, [],
                               attach_id="add-again", want=[idx])
        assert got is not None and got.placeholders[0].name == ph
        await asyncio.sleep(0.6)
        await svc.lease.sweep()
        await asyncio.sleep(0.1)
        assert lc.cluster.get("gpu-pool", ph) is not None and svc.lease.expired == 0
    run(body, worker_overrides={"warm_pool_size": 1})


def test_a_lease_granted_to_part_of_an_entire_mount_group_ends_the_whole_group():
    """An entire mount from the warm pool is a group of 1-GPU placeholders. A worker killed
    while granting its lease leaves the annotation on some of them only; the successor's
    expiry then asked to remove part of an entire mount, which is refused, and the lease was
    retried for 30 s and more while its GPUs stayed attached (chaos seed rpl150). The whole
    group goes when any part of it expires."""
    async def body(lc):
        w = lc.nodes["node-0"].worker
        svc = w.service
        for _ in range(200):
            if len(w.pool.standby()) >= 3:
                break
            await asyncio.sleep(0.01)
        lc.tenant("t")
        code, b = await lc.add("default", "t", 3, entire=True)
        assert code == 200 and len(b["devices"]) == 3
        names = sorted({d["placeholder"] for d in b["devices"]})
        assert len(names) == 3                              # a group of pool placeholders
        past = str(time.time() - 1)
        for n in names[:2]:                                 # the grant reached two of three
            lc.cluster.patch("gpu-pool", n, {"metadata": {"annotations": {ANN_LEASE: past}}})

        async def gone():
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            return not st.hot
        await asyncio.sleep(0.05)                           # the watch delivers the patch
        await svc.lease.expire_owner("default", "t")
        assert await until(gone, 2.0)
        assert not await lc.audit("default", "t")
    run(body, worker_overrides={"warm_pool_size": 3})


def _writes(lc):
    v = lc.cluster.requests_by_verb
    return {k: v.get(k, 0) for k in ("POST", "PATCH", "DELETE")}


def _count(before, after):
    return {k: after[k] - before[k] for k in after}


@pytest.mark.parametrize("mode", ["plain", "pool", "dra", "trim"])
def test_a_leased_attach_writes_no_more_than_an_unleased_one(mode):
    """The lease travels in the booking itself (placeholder POST, pool claim PATCH, the DRA
    placeholder): no write is added for it (round 4: one PATCH per placeholder after the
    mount, and a crash window between "GPU granted" and "lease recorded")."""
    kw = {"worker_overrides": {}}
    if mode == "pool":
        kw["worker_overrides"]["warm_pool_size"] = 4
    if mode == "dra":
        kw["gpu_api"] = "dra"
    if mode == "trim":
        kw["worker_overrides"]["placement_enforce"] = "trim"

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        if mode == "pool":
            await svc.ph.informer.wait_for(lambda: len(svc.pool.standby()) >= 4, 10)
        counts = {}
        for lease in ("", "3600"):
            await asyncio.sleep(0.05)
            before = _writes(lc)
            code, b = await lease_add(lc, "default", "t", 2, lease) if lease else \
                await lc.add("default", "t", 2)
            assert code == 200, b
            counts[lease] = _count(before, _writes(lc))
            leased = [p for p in lc.cluster.placeholders()
                      if (p["metadata"].get("annotations") or {}).get(
                          "gpumounter.amd.com/owner-name") == "t"
                      and (p["metadata"].get("annotations") or {}).get(ANN_LEASE)]
            assert len(leased) == (2 if lease else 0), leased
            code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
            assert code == 200
            if mode == "pool":
                await svc.ph.informer.wait_for(lambda: len(svc.pool.standby()) >= 4, 10)
        assert counts["3600"] == counts[""], counts
    run(body, **kw)


@pytest.mark.parametrize("pool", [0, 2])
def test_a_worker_killed_between_booking_and_mount_leaves_no_unleased_placeholder(pool):
    """GM_FAULT=cgroup_rule:1:exit: the worker process dies (as under SIGKILL) after its
    placeholders are booked and admitted, before anything is mounted. Every placeholder the
    attach booked already carries the lease; the next worker finishes the attach on the
    client's retry (same idempotency key) and the lease ends it on time."""
    import json as _json

    from gpumounter_amd.fakes.deployment import ProcessCluster

    with ProcessCluster(worker_env={"GM_FAULT": "cgroup_rule:1.0:exit",
                                    "GM_WARM_POOL_SIZE": str(pool)}) as pc:
        pc.tenant("t")
        if pool:
            end = time.time() + 20
            while time.time() < end and sum(
                    1 for p in pc.placeholders()
                    if (p["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/mount-mode") == "standby") < pool:
                time.sleep(0.05)
        q = "/addgpu/namespace/default/pod/t/gpu/2/isEntireMount/false?lease=2"
        code, body = pc._master("GET", q, headers={"Accept": "application/json",   # noqa: SLF001
                                                   "Idempotency-Key": "K1"})
        assert code == 500, body
        assert pc.procs["worker-node-0"].wait(10) == 137
        mine = [p for p in pc.placeholders()
                if (p["metadata"].get("annotations") or {}).get(
                    "gpumounter.amd.com/owner-name") == "t"]
        assert mine, "the booking happened before the crash"
        assert all((p["metadata"].get("annotations") or {}).get(ANN_LEASE) for p in mine), \
            [p["metadata"]["annotations"] for p in mine]
        # a worker without the fault: the client's retry replays the attach with its lease
        pc._worker_env["node-0"].pop("GM_FAULT")                    # noqa: SLF001
        pc.restart_worker("node-0")
        end = time.time() + 10
        while True:          # until the master's worker watch has the new address
            code, body = pc._master("GET", q, headers={                        # noqa: SLF001
                "Accept": "application/json", "Idempotency-Key": "K1"})
            if code == 200 or time.time() > end:
                break
            time.sleep(0.1)
        assert code == 200, body
        body = _json.loads(body)
        assert len(body["devices"]) == 2
        end = time.time() + 10
        left = None
        while time.time() < end:
            left = [p for p in pc.placeholders()
                    if (p["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/owner-name") == "t"
                    and (p["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/mount-mode") != "standby"]
            if not left:
                break
            time.sleep(0.1)
        assert not left, "the lease never ended the attach"
        assert pc.audit("default", "t") == []


def test_an_expiry_that_keeps_failing_tells_the_pod():
    """a RemoveGPU refusal that does not go away (here GPUNotFound on every try)
    was retried every lease_retry_s with only ERROR logs; after the quick retries the Pod now
    gets a GPULeaseExpired warning Event naming the failure (once), and retries continue."""
    from gpumounter_amd.api import gpu_mount as api

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        svc.lease.ERROR_RETRY_S = (0.05, 0.05, 0.05)
        calls = []

        async def refuse(req):
            calls.append(req)
            return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_GPU_NOT_FOUND)
        code, b = await lease_add(lc, "default", "t", 1, 0.1)
        assert code == 200, b
        real = svc.remove_gpu
        svc.remove_gpu = refuse

        async def warned():
            return any(e["reason"] == "GPULeaseExpired" and e["type"] == "Warning" and
                       "could not be detached" in e["message"]
                       for e in lc.cluster.events_for("default", "t"))
        assert await until(warned, timeout=5.0), lc.cluster.events_for("default", "t")
        assert len(calls) >= 4
        n = sum(1 for e in lc.cluster.events_for("default", "t")
                if "could not be detached" in e["message"])
        assert n == 1
        svc.remove_gpu = real
    run(body, worker_overrides={"lease_retry_s": 0.2})


def test_a_slow_attach_gets_its_whole_lease():
    """the lease is booked when the request arrives; an attach that waits long for
    admission must not spend its lease in that wait. Past LEASE_REBASE_S the lease starts at
    the mount (and the reply says so)."""
    from gpumounter_amd.fakes.apiserver import LatencyModel

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        t0 = time.time()
        code, b = await lease_add(lc, "default", "t", 1, 2.0)    # admission alone takes 1.5 s
        t1 = time.time()
        assert code == 200 and t1 - t0 >= 1.5
        (p,) = [p for p in lc.cluster.placeholders()
                if (p["metadata"].get("annotations") or {}).get(ANN_LEASE)]
        until_ = float(p["metadata"]["annotations"][ANN_LEASE])
        assert until_ >= t1 + 1.8, (until_ - t1)            # counted from the mount, not t0
        await asyncio.sleep(1.0)                            # past t0 + 2 s: still attached
        st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
        assert len(st.hot) == 1

        async def gone():
            st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
            return not st.hot
        assert await until(gone, 5.0)
    run(body, latency=LatencyModel(schedule_ms=1500.0))
