"""Detach ends at the DELETE's answer, not at the watch's echo of it.

A grace-0 placeholder DELETE answered 200/404 means the object is gone from the apiserver and
from the scheduler's books (the reference's detach likewise ends at NotFound:
/root/reference/pkg/util/gpu/allocator/allocator.go:284-317). The worker tombstones the UID and
answers; every later view leaves the tombstoned placeholder out. These tests hold every watch
event back by 1 s and re-attach at once: the second attach must see the released GPU as free
and the Pod's ownership exactly as the apiserver has it, and the late DELETED echo must not be
mistaken for a foreign delete."""
import asyncio
import time

import pytest

from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.models.device import normalize_device_id


def _owned(lc, pod):
    return sorted(p["metadata"]["name"] for p in lc.cluster.placeholders()
                  if (p["metadata"].get("annotations") or {}).get(
                      "gpumounter.amd.com/owner-name") == pod
                  and (p["metadata"].get("annotations") or {}).get(
                      "gpumounter.amd.com/mount-mode") not in ("standby",))


@pytest.mark.parametrize("pool", [0, 3])
def test_reattach_right_after_detach_with_a_slow_watch(pool):
    async def main():
        async with LocalCluster(cgroup_mode="v2",
                                worker_overrides={"warm_pool_size": pool}) as lc:
            lc.tenant("t")
            svc = lc.nodes["node-0"].worker.service
            if pool:
                await svc.ph.informer.wait_for(lambda: len(svc.pool.standby()) >= pool, 10)
            code, b = await lc.add("default", "t", 2)
            assert code == 200, b
            a_dev, b_dev = b["devices"]
            lc.cluster.watch_delay_s = 1.0            # every watch event from now on: +1 s
            t0 = time.monotonic()
            code, r = await lc.remove("default", "t", [a_dev["uuid"]])
            took = time.monotonic() - t0
            assert code == 200, r
            assert took < 0.5, f"detach waited {took:.2f}s (for the watch echo?)"
            # the worker's view right away: the removed GPU is free, the kept one is not
            pod = lc.cluster.get("default", "t")
            st = await svc.pod_state(pod)
            hot = {g.bdf for g in st.hot}
            assert hot == {b_dev["bdf"]}
            free = {g.bdf for g in svc._free(st)}          # noqa: SLF001
            # with the warm pool the GPU may have gone back to it (a standby: claimable)
            keys = svc.inv.by_key()
            standby = {keys[normalize_device_id(d)].bdf for ph in
                       (svc.pool.standby() if pool else []) for d in ph.device_ids}
            assert a_dev["bdf"] in free | standby and b_dev["bdf"] not in free | standby
            # re-attach at once, still ahead of every echo
            t1 = time.monotonic()
            code, c = await lc.add("default", "t", 1)
            assert code == 200, c
            new = c["devices"][0]["bdf"]
            assert new != b_dev["bdf"]
            st = await svc.pod_state(lc.cluster.get("default", "t"))
            assert sorted(g.bdf for g in st.hot) == sorted([b_dev["bdf"], new])
            # the apiserver agrees: two placeholders of the Pod, holding exactly those GPUs
            assert len(_owned(lc, "t")) == 2
            node = lc.nodes["node-0"].node
            held = {normalize_device_id(d) for d, (ns, p, _) in node.allocated.items()
                    if p in _owned(lc, "t")}
            assert held == {normalize_device_id(b_dev["bdf"]), normalize_device_id(new)}
            # the echoes arrive: nothing is revoked, the node matches the ledger
            await asyncio.sleep(max(0.0, 1.3 - (time.monotonic() - t1)))
            lc.cluster.watch_delay_s = 0.0
            await asyncio.sleep(0.3)
            assert not await lc.audit("default", "t")
            st = await svc.pod_state(lc.cluster.get("default", "t"))
            assert sorted(g.bdf for g in st.hot) == sorted([b_dev["bdf"], new])
            assert lc.nodes["node-0"].worker.metrics.reconcile_actions.labels(
                action="revoke")._value.get() == 0
    asyncio.run(main())


def test_detach_makes_one_apiserver_write_and_no_watch_wait():
    """The default detach path: one DELETE, answered; no GET and no wait in between."""
    async def main():
        async with LocalCluster(cgroup_mode="v2") as lc:
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)
            assert code == 200
            before = dict(lc.cluster.requests_by_verb)
            lc.cluster.watch_delay_s = 2.0
            t0 = time.monotonic()
            code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
            assert code == 200 and time.monotonic() - t0 < 0.5
            after = lc.cluster.requests_by_verb
            delta = {k: after.get(k, 0) - before.get(k, 0) for k in after
                     if after.get(k, 0) != before.get(k, 0)}
            assert delta.get("DELETE") == 1 and not delta.get("GET"), delta
            lc.cluster.watch_delay_s = 0.0
    asyncio.run(main())
