"""GPU hot-mount on clusters whose GPUs come from a DRA driver (``gpu_allocation=dra``):
placeholders hold ResourceClaims pinned to the topology-chosen devices by a CEL selector, the
worker's ledger is read from ResourceClaims + the node's ResourceSlice (gpumounter_amd/node/dra.py),
the kubelet's device manager knows nothing about the GPUs. Hermetic control plane: fakes/dra.py
(its scheduler/driver parity with a real cluster is unpinned — no cluster here)."""
import asyncio
import time

import pytest

from gpumounter_amd.cluster.placeholder import ANN_GPUS
from gpumounter_amd.fakes.dra import parse_selector
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.utils.config import Config


def run(coro_fn, **kw):
    async def main():
        async with LocalCluster(gpu_api="dra", **kw) as lc:
            return await coro_fn(lc)
    return asyncio.run(main())


def claims(lc):
    return dict(lc.cluster.dra.claims)


def allocated_bdfs(claim):
    alloc = (claim.get("status") or {}).get("allocation") or {}
    return [r["device"] for r in alloc.get("devices", {}).get("results", [])]


async def until(pred, timeout=5.0):
    t0 = time.monotonic()
    while not pred():
        assert time.monotonic() - t0 < timeout
        await asyncio.sleep(0.01)


def test_dra_attach_detach_pins_devices_with_claims():
    async def body(lc):
        node = lc.nodes["node-0"].node
        lc.tenant("t")
        code, b = await lc.add("default", "t", 2)
        assert code == 200, b
        got = sorted(d["bdf"] for d in b["devices"]) if "bdf" in b["devices"][0] else None
        phs = lc.cluster.placeholders()
        assert len(phs) == 2
        by_idx = {f"gpu-{g.index}": g.bdf for g in node.gpus}
        held = []
        for p in phs:
            c = p["spec"]["containers"][0]["resources"]
            assert "limits" not in c and c["claims"] == [{"name": "gpus"}]
            assert p["metadata"]["annotations"][ANN_GPUS] == "1"
            name = p["spec"]["resourceClaims"][0]["resourceClaimName"]
            claim = lc.cluster.dra.claims[(p["metadata"]["namespace"], name)]
            devs = [by_idx[d] for d in allocated_bdfs(claim)]
            sel = claim["spec"]["devices"]["requests"][0]["exactly"]["selectors"][0]
            _, attr, vals = parse_selector(sel["cel"]["expression"])
            assert attr == "pciAddr" and vals == devs      # the scheduler took exactly those
            assert claim["status"]["reservedFor"][0]["uid"] == p["metadata"]["uid"]
            held += devs
        if got is not None:
            assert sorted(held) == got
        assert not await lc.audit("default", "t")
        assert not node.write_checkpoint                     # device manager not involved
        ledger = lc.nodes["node-0"].worker.ledger
        assert ledger.api_version == "resource.k8s.io/v1"
        # the claims' allocation came with the claim watch, not a GET per placeholder
        assert ledger.claim_cache_hits >= 1
        code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
        assert code == 200
        assert not await lc.audit("default", "t")
        await until(lambda: not claims(lc))                  # claims deleted after the pods
        assert node.allocated == {}
    run(body)


@pytest.mark.parametrize("entire", [True, False])
def test_dra_insufficient_is_all_or_nothing(entire):
    async def body(lc):
        lc.tenant("big")
        code, text = await lc.add("default", "big", 9, entire=entire, accept_json=False)
        assert (code, text) == (500, "Insufficient GPU on Node: node-0\n")
        await until(lambda: not lc.cluster.placeholders() and not claims(lc))
        assert lc.nodes["node-0"].node.allocated == {}
    run(body)


def test_dra_entire_mount_is_one_claim_of_n_devices():
    async def body(lc):
        lc.tenant("e")
        code, b = await lc.add("default", "e", 4, entire=True)
        assert code == 200 and len(b["devices"]) == 4
        (claim,) = claims(lc).values()
        ex = claim["spec"]["devices"]["requests"][0]["exactly"]
        assert ex["count"] == 4 and len(allocated_bdfs(claim)) == 4
        assert (await lc.add("default", "e", 1))[0] == 500        # entire: no more adds
        assert (await lc.remove("default", "e", [d["uuid"] for d in b["devices"]]))[0] == 200
        await until(lambda: not claims(lc))
    run(body)


def test_dra_stale_preference_retries_unpinned():
    """The topology choice came from a ledger view that is stale: the pinned claim cannot be
    allocated, so the reservation is retried once without the selector."""
    async def body(lc):
        node = lc.nodes["node-0"].node
        svc = lc.nodes["node-0"].worker.service
        # someone else's claim holds GPU 0 (a DRA workload pod)
        lc.cluster.dra.create("default", {"metadata": {"name": "other"}, "spec": {"devices": {
            "requests": [{"name": "g", "exactly": {"deviceClassName": "gpu.amd.com", "count": 1,
                          "selectors": [{"cel": {"expression":
                              f'device.attributes["gpu.amd.com"].pciAddr == '
                              f'"{node.gpus[0].bdf}"'}}]}}]}}})
        lc.cluster.create_pod("default", {
            "metadata": {"name": "other"},
            "spec": {"resourceClaims": [{"name": "g", "resourceClaimName": "other"}],
                     "containers": [{"name": "c", "image": "x:1",
                                     "resources": {"claims": [{"name": "g"}]}}]}})
        await until(lambda: allocated_bdfs(lc.cluster.dra.claims[("default", "other")]))
        svc._preferred = lambda n, st, free=None: [node.gpus[0].bdf]   # stale view
        lc.tenant("t")
        code, b = await lc.add("default", "t", 1)
        assert code == 200, b
        mine = [c for (ns, n), c in claims(lc).items() if n != "other"]
        assert len(mine) == 1
        assert "selectors" not in mine[0]["spec"]["devices"]["requests"][0]["exactly"]
        assert allocated_bdfs(mine[0]) != ["gpu-0"]
        assert not await lc.audit("default", "t")
    run(body)


def test_dra_worker_restart_recovers_from_claims():
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        await lc.stop_worker("node-0")
        await lc.start_worker("node-0")
        w = lc.nodes["node-0"].worker
        want = f"127.0.0.1:{w.grpc_port}"
        await lc.master.workers.informer.wait_for(
            lambda: lc.master.workers.target("node-0") == want, 10)
        st = await w.service.pod_state(lc.cluster.get("default", "t"))
        assert sorted(g.uuid for g in st.hot) == sorted(d["uuid"] for d in b["devices"])
        assert (await lc.remove("default", "t", [d["uuid"] for d in b["devices"]]))[0] == 200
        await until(lambda: not claims(lc))
    run(body)


def test_dra_warm_pool_standby_claims():
    async def body(lc):
        pool = lc.nodes["node-0"].worker.pool
        await until(lambda: len(pool.standby()) == 4)
        assert len(claims(lc)) == 4
        for p in lc.cluster.placeholders():
            assert p["spec"]["resourceClaims"][0]["resourceClaimName"] == p["metadata"]["name"]
        lc.tenant("t")
        standby_uids = {p.uid for p in pool.standby()}
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        # both GPUs come from claimed standby placeholders (a metadata PATCH, no create); the
        # pool's refill creating new standby placeholders meanwhile is not part of the attach
        # (counting POSTs raced with it under load)
        owned = lc.nodes["node-0"].worker.service.ph.owned_by(lc.cluster.get("default", "t"))
        assert {p["metadata"]["uid"] for p in owned} <= standby_uids and len(owned) == 2
        assert not await lc.audit("default", "t")
        assert (await lc.remove("default", "t", [d["uuid"] for d in b["devices"]]))[0] == 200
        await until(lambda: len(pool.standby()) == 4)
    run(body, worker_overrides={"warm_pool_size": 4})


def test_dra_ledger_ignores_other_drivers_and_nodes():
    async def body(lc):
        led = lc.nodes["node-0"].worker.ledger
        assert len(await led.allocatable()) == len(lc.nodes["node-0"].node.gpus)
        foreign = {"metadata": {"name": "f", "namespace": "x"},
                   "status": {"allocation": {"devices": {"results": [
                       {"request": "r", "driver": "other.example.com", "pool": "node-0",
                        "device": "gpu-0"},
                       {"request": "r", "driver": "gpu.amd.com", "pool": "node-9",
                        "device": "gpu-0"}]}},
                       "reservedFor": [{"resource": "pods", "name": "p", "uid": "u"}]}}
        assert await led.claim_devices(foreign) == []
    run(body, n_nodes=1)


def test_dra_config_validation():
    with pytest.raises(ValueError):
        Config.load(env={}, gpu_allocation="dra", device_plugin=True)
    with pytest.raises(ValueError):
        Config.load(env={}, gpu_allocation="cdi")
    assert Config.load(env={"GM_GPU_ALLOCATION": "dra"}).gpu_allocation == "dra"


def test_dra_reconciler_deletes_orphan_claims():
    """A worker that died between creating a placeholder's claim and its Pod leaves a claim
    that holds nothing; the reconciler deletes it (after its grace), and only ours."""
    async def body(lc):
        w = lc.nodes["node-0"].worker
        lc.tenant("t")
        code, b = await lc.add("default", "t", 1)
        assert code == 200
        body_ = w.placeholders.build(lc.cluster.get("default", "t"), 1, "single")
        orphan = w.placeholders.claim_for(body_)
        await w.kube.create_claim(orphan["metadata"]["namespace"], orphan)
        lc.cluster.dra.create("default", {"metadata": {"name": "not-ours"}, "spec": {
            "devices": {"requests": [{"name": "g", "exactly": {
                "deviceClassName": "gpu.amd.com", "count": 1}}]}}})
        rec = w.reconciler
        rec.stuck_after_s = 3600
        assert (await rec.run_once()).claims_deleted == []        # still in its grace
        rec.stuck_after_s = 0
        rep = await rec.run_once()
        assert rep.claims_deleted == [f"{orphan['metadata']['namespace']}/"
                                      f"{orphan['metadata']['name']}"]
        left = {n for (_, n) in claims(lc)}
        assert "not-ours" in left and orphan["metadata"]["name"] not in left
        assert len(left) == 2                                      # the live attach's claim
        assert not await lc.audit("default", "t")
    run(body)


def test_doctor_checks_resource_slices_in_dra_mode():
    from gpumounter_amd.utils import doctor

    async def main():
        async with LocalCluster(gpu_api="dra", start_master=False, start_workers=False) as lc:
            cfg = Config.load(env={}, amdsmi_lib="mock", kube_api=lc.api_url,
                              node_name="node-0", gpu_allocation="dra",
                              cgroup_root="/nonexistent", systemd_device_allow="off")
            good = await asyncio.get_running_loop().run_in_executor(None, doctor.run, cfg)
            cfg2 = Config.load(env={}, amdsmi_lib="mock", kube_api=lc.api_url,
                               node_name="node-0", gpu_allocation="dra",
                               dra_driver="other.example.com", cgroup_root="/nonexistent",
                               systemd_device_allow="off")
            bad = await asyncio.get_running_loop().run_in_executor(None, doctor.run, cfg2)
            return good, bad
    good, bad = asyncio.run(main())
    g = {c.name: c for c in good}["dra"]
    assert g.status == "ok" and "8 gpu.amd.com device(s)" in g.detail, g
    assert {c.name: c for c in bad}["dra"].status == "fail"


def test_dra_tenant_namespace_mode():
    """Placeholders (and so their claims) in the tenant's namespace: the claim watch covers
    every namespace through the node label."""
    async def body(lc):
        lc.tenant("t", ns="team-a")
        code, b = await lc.add("team-a", "t", 2)
        assert code == 200, b
        assert {ns for (ns, _) in claims(lc)} == {"team-a"}
        assert lc.nodes["node-0"].worker.ledger.claim_cache_hits >= 2
        assert not await lc.audit("team-a", "t")
        assert (await lc.remove("team-a", "t", [d["uuid"] for d in b["devices"]]))[0] == 200
        await until(lambda: not claims(lc))
    run(body, placeholder_namespace_mode="tenant")


@pytest.mark.parametrize("mode", ["pool", "tenant"])
def test_dra_device_class_quota(mode):
    """ResourceQuota ``gpu.amd.com.deviceclass.resource.k8s.io/devices`` caps hot-mounted GPUs:
    enforced by the worker for pool-namespace placeholders, by the apiserver's quota admission
    of the claims in tenant mode; the refusal is a 403 QuotaExceeded either way."""
    key = "gpu.amd.com.deviceclass.resource.k8s.io/devices"

    async def body(lc):
        lc.cluster.set_quota("team-a", "gpus", {key: "3"})
        lc.cluster.dra.create("team-a", {"metadata": {"name": "own"}, "spec": {"devices": {
            "requests": [{"name": "g", "exactly": {"deviceClassName": "gpu.amd.com",
                                                   "count": 1}}]}}})   # the tenant's own GPU
        lc.tenant("p1", ns="team-a")
        lc.tenant("other", ns="team-b")
        code, b1 = await lc.add("team-a", "p1", 1)
        assert code == 200, b1
        code, b = await lc.add("team-a", "p1", 2)
        assert code == 403 and "exceeded quota" in b["message"], b
        assert len(claims(lc)) == 2           # the refused attach left no claim behind
        code, b2 = await lc.add("team-a", "p1", 1)                 # 1 own + 2 = 3 = hard
        assert code == 200, b2
        assert (await lc.add("team-a", "p1", 1))[0] == 403
        assert (await lc.add("team-b", "other", 3))[0] == 200      # no quota there
        assert not await lc.audit("team-a", "p1")
    run(body, placeholder_namespace_mode=mode)


def test_dra_tenant_own_claim_gpus_are_not_removable():
    """A Pod that got a GPU through its own ResourceClaim: hot-mounts go to other GPUs, and its
    own GPU can never be removed (reference allocator.go:112-123)."""
    async def body(lc):
        node = lc.nodes["node-0"].node
        lc.cluster.dra.create("default", {"metadata": {"name": "own"}, "spec": {"devices": {
            "requests": [{"name": "g", "exactly": {"deviceClassName": "gpu.amd.com",
                                                   "count": 1}}]}}})
        lc.cluster.create_pod("default", {
            "metadata": {"name": "t"},
            "spec": {"resourceClaims": [{"name": "g", "resourceClaimName": "own"}],
                     "containers": [{"name": "main", "image": "x:1",
                                     "resources": {"claims": [{"name": "g"}]}}]}})
        await until(lambda: (lc.cluster.get("default", "t") or {}).get("status", {})
                    .get("phase") == "Running")
        (own,) = [by for by in allocated_bdfs(lc.cluster.dra.claims[("default", "own")])]
        own_bdf = next(g.bdf for g in node.gpus if f"gpu-{g.index}" == own)
        svc = lc.nodes["node-0"].worker.service
        st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
        assert [g.bdf for g in st.own] == [own_bdf]
        code, b = await lc.add("default", "t", 2)
        assert code == 200, b
        assert own_bdf not in [d["bdf"] for d in b["devices"]]
        own_uuid = next(g.uuid for g in node.gpus if g.bdf == own_bdf)
        code, text = await lc.remove("default", "t", [own_uuid], accept_json=False)
        assert (code, text) == (400, "Invalid UUIDs: " + own_uuid + "\n")
        assert not await lc.audit("default", "t")
    run(body)


def test_dra_a_standby_created_behind_a_failed_reply_keeps_its_claim():
    """The pool's create of a standby placeholder can fail after it happened (reply lost, the
    retry meets 409 because an attach already claimed the new placeholder and changed it). Its
    ResourceClaim then holds that attach's GPU: deleting it as the failed create's leftover took
    the GPU from the ledger under the mounted Pod (chaos: DRA + warm pool 3 + leases, seed 83)."""
    from gpumounter_amd.cluster.kube import Conflict

    async def body(lc):
        pool = lc.nodes["node-0"].worker.pool
        await until(lambda: len(pool.standby()) == 1)
        kube = pool.ph.kube
        real_create = kube.create_pod
        made = []

        async def create(ns, pod):
            out = await real_create(ns, pod)
            made.append(out["metadata"]["name"])
            raise Conflict(409, f'pods "{out["metadata"]["name"]}" already exists')
        kube.create_pod = create
        pool.target = 2
        await pool.refill()
        kube.create_pod = real_create
        assert made and ("gpu-pool", made[0]) in claims(lc)    # the Pod exists: its claim stays
        assert lc.cluster.get("gpu-pool", made[0]) is not None
    run(body, worker_overrides={"warm_pool_size": 1})
