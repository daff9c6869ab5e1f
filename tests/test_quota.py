"""Namespace GPU quotas apply to hot-mounted GPUs (gpumounter_amd/cluster/quota.py).

Pool-namespace placeholders are charged to the pool namespace by Kubernetes itself, so the
worker enforces the tenant namespace's ``requests.amd.com/gpu`` quota; with tenant-namespace
placeholders the (fake) apiserver's quota admission does, and the refusal is mapped the same way.
"""
import asyncio

import pytest

from gpumounter_amd.fakes.harness import LocalCluster


def run(coro_fn, **kw):
    async def main():
        async with LocalCluster(**kw) as lc:
            return await coro_fn(lc)
    return asyncio.run(main())


@pytest.mark.parametrize("mode", ["pool", "tenant"])
def test_quota_caps_hot_mounted_gpus_per_namespace(mode):
    async def body(lc):
        lc.cluster.set_quota("team-a", "gpus", {"requests.amd.com/gpu": "3"})
        lc.tenant("own", ns="team-a", gpus=1)        # its own GPU counts against the quota
        lc.tenant("p1", ns="team-a")
        lc.tenant("p2", ns="team-a")
        lc.tenant("other", ns="team-b")
        code, b1 = await lc.add("team-a", "p1", 1)
        assert code == 200, b1
        code, b = await lc.add("team-a", "p2", 2)
        assert code == 403, b
        assert "exceeded quota" in b["message"] and "gpus" in b["message"]
        code, b2 = await lc.add("team-a", "p2", 1)   # 1 own + 2 hot = 3 = hard
        assert code == 200, b2
        assert (await lc.add("team-a", "p1", 1))[0] == 403
        assert (await lc.add("team-b", "other", 3))[0] == 200   # another namespace: no quota
        code, _ = await lc.remove("team-a", "p1", [b1["devices"][0]["uuid"]])
        assert code == 200
        assert (await lc.add("team-a", "p1", 1))[0] == 200       # room again after detach
        svc = lc.nodes["node-0"].worker.service
        await svc.notify.drain()
        assert any(e["reason"] == "GPUAttachFailed" and "exceeded quota" in e["message"]
                   for e in lc.cluster.events_for("team-a", "p2"))
        for p in ("p1", "p2"):
            assert await lc.audit("team-a", p) == []
    run(body, placeholder_namespace_mode=mode)


def test_quota_text_reply_and_off_switch():
    async def body(lc):
        lc.cluster.set_quota("default", "gpus", {"requests.amd.com/gpu": "1"})
        lc.tenant("t")
        assert (await lc.add("default", "t", 1))[0] == 200
        code, text = await lc.add("default", "t", 1, accept_json=False)
        assert code == 403 and text.startswith("QuotaExceeded: exceeded quota: gpus")
    run(body)

    async def body_off(lc):
        lc.cluster.set_quota("default", "gpus", {"requests.amd.com/gpu": "1"})
        lc.tenant("t")
        assert (await lc.add("default", "t", 2))[0] == 200
    run(body_off, worker_overrides={"quota_mode": "off"})


def test_concurrent_attaches_never_exceed_the_quota():
    async def body(lc):
        lc.cluster.set_quota("default", "gpus", {"requests.amd.com/gpu": "2"})
        for i in range(4):
            lc.tenant(f"t{i}")
        res = await asyncio.gather(*[lc.add("default", f"t{i}", 1) for i in range(4)])
        codes = sorted(c for c, _ in res)
        assert codes == [200, 200, 403, 403], res
        held = sum(1 for p in lc.cluster.placeholders()
                   if not p["metadata"].get("deletionTimestamp"))
        assert held == 2
    run(body)


def test_recheck_rolls_back_an_overshoot_from_another_node():
    """Two workers (nodes) attach into one namespace at once: the per-node lock cannot see the
    other node, the post-create recheck can — the quota is never exceeded."""
    async def body(lc):
        lc.cluster.set_quota("default", "gpus", {"requests.amd.com/gpu": "1"})
        lc.tenant("a", node="node-0")
        lc.tenant("b", node="node-1")
        res = await asyncio.gather(lc.add("default", "a", 1), lc.add("default", "b", 1))
        ok = [c for c, _ in res if c == 200]
        assert len(ok) <= 1, res
        assert all(c in (200, 403) for c, _ in res), res

        async def settled():
            live = [p for p in lc.cluster.placeholders()
                    if not p["metadata"].get("deletionTimestamp")]
            return len(live) == len(ok)
        for _ in range(200):
            if await settled():
                break
            await asyncio.sleep(0.01)
        assert await settled()
    run(body, n_nodes=2)


def test_placement_correction_within_a_tight_tenant_quota_keeps_the_plugins_choice():
    """Tenant-namespace placeholders: the quota admits exactly the request, so the correction's
    extra holds are refused by the apiserver's quota admission. The attach still succeeds with
    the GPUs the plugin chose (valid, worse placed) instead of failing."""
    async def body(lc):
        lc.cluster.set_quota("team-a", "gpus", {"requests.amd.com/gpu": "2"})
        lc.tenant("other", ns="team-b")
        lc.tenant("t", ns="team-a")
        assert (await lc.add("team-b", "other", 3))[0] == 200          # GPUs 0, 1, 2
        code, b = await lc.add("team-a", "t", 2)
        assert code == 200, b
        assert sorted(d["index"] for d in b["devices"]) == [3, 4]      # across the sockets
        assert await lc.audit("team-a", "t") == []
        assert len(lc.nodes["node-0"].node.allocated) == 5
    run(body, placeholder_namespace_mode="tenant", alloc_policy="first-free")


def test_trim_mode_within_a_tight_tenant_quota_falls_back_to_a_plain_reservation():
    async def body(lc):
        lc.cluster.set_quota("team-a", "gpus", {"requests.amd.com/gpu": "2"})
        lc.tenant("t", ns="team-a")
        code, b = await lc.add("team-a", "t", 2)
        assert code == 200, b
        assert await lc.audit("team-a", "t") == []
        assert (await lc.add("team-a", "t", 1))[0] == 403               # the quota itself holds
    run(body, placeholder_namespace_mode="tenant", alloc_policy="first-free",
        worker_overrides={"placement_enforce": "trim"})
