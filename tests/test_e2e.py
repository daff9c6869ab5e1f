"""End-to-end behaviour through the real master HTTP API → worker gRPC → C++ node ops, on the
hermetic control plane (reference behaviour table: SURVEY §2.5; defects fixed: §2.6)."""
import asyncio
import os
import subprocess

import pytest

from gpumounter_amd import _native
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.models.types import LABEL_OWNER
from gpumounter_amd.node import checkpoint as ckpt


def run(coro_fn, **kw):
    async def main():
        async with LocalCluster(**kw) as lc:
            return await coro_fn(lc)
    return asyncio.run(main())


def node_of(lc):
    return lc.nodes["node-0"].node


async def text_get(lc, path):
    async with lc.session.get(lc.master_url + path) as r:
        return r.status, await r.text()


# ------------------------------------------------------------------------------ HTTP contract
def test_reference_text_contract_success_path():
    async def body(lc):
        lc.tenant("gpu-pod")
        assert await text_get(lc, "/") == (200, "This is gpu mounter api!\n")
        code, text = await lc.add("default", "gpu-pod", 2, accept_json=False)
        assert (code, text) == (200, "Add GPU Success\n")
        # the reference QuickStart's curl: repeated urlencoded uuids, force=1
        st = await lc.nodes["node-0"].worker.service.pod_state(lc.cluster.get("default",
                                                                              "gpu-pod"))
        uuids = [g.uuid for g in st.hot]
        code, text = await lc.remove("default", "gpu-pod", uuids, force=True, accept_json=False)
        assert (code, text) == (200, "Remove GPU Success\n")
    run(body)


@pytest.mark.parametrize("path,code,text", [
    ("/addgpu/namespace/default/pod/p/gpu/abc/isEntireMount/false", 400,
     "Invalid param gpuNum: abc\n"),
    ("/addgpu/namespace/default/pod/p/gpu/1/isEntireMount/yes", 400,
     "Invalid param isEntireMount: yes(should be true or false)\n"),
    ("/addgpu/namespace/default/pod/p/gpu/99999999999/isEntireMount/false", 400,
     "Invalid param gpuNum: 99999999999\n"),
    ("/addgpu/namespace/default/pod/p/gpu/0/isEntireMount/true", 400,
     "Invalid param gpuNum: 0\n"),                    # reference: worker divide-by-zero panic
    ("/addgpu/namespace/default/pod/nope/gpu/1/isEntireMount/T", 404,
     "No pod: nope in namespace: default\n"),
])
def test_add_parameter_validation(path, code, text):
    async def body(lc):
        lc.tenant("p")
        assert await text_get(lc, path) == (code, text)
    run(body)


def test_remove_parameter_validation():
    async def body(lc):
        lc.tenant("p")
        code, text = await lc.remove("default", "p", [], accept_json=False)
        assert (code, text) == (400, "Invalid parameter\n")
        async with lc.session.post(lc.master_url + "/removegpu/namespace/default/pod/p/force/x",
                                   data={"uuids": "u"}) as r:
            assert (r.status, await r.text()) == (
                400, "Invalid parameter force: x(should be true or false)\n")
        code, text = await lc.remove("default", "ghost", ["u"], accept_json=False)
        assert (code, text) == (404, "No pod: ghost in namespace: default\n")
        code, text = await lc.remove("default", "p", ["bogus"], accept_json=False)
        assert (code, text) == (400, "Invalid UUIDs: bogus\n")
    run(body)


@pytest.mark.parametrize("entire", [True, False])
def test_insufficient_gpus_is_all_or_nothing(entire):
    async def body(lc):
        lc.tenant("big")
        code, text = await lc.add("default", "big", 9, entire=entire, accept_json=False)
        assert (code, text) == (500, "Insufficient GPU on Node: node-0\n")
        await asyncio.sleep(0.05)
        assert lc.cluster.placeholders() == []          # rollback deleted every placeholder
        assert node_of(lc).allocated == {}
        assert not await lc.audit("default", "big")
    run(body)


# ------------------------------------------------------------------------------ policy
def test_mount_policy_matches_reference_can_mount():
    async def body(lc):
        lc.tenant("e")
        lc.tenant("s")
        assert (await lc.add("default", "e", 2, entire=True))[0] == 200
        code, b = await lc.add("default", "e", 1)              # entire → no more adds
        assert code == 500 and "policy" in b["error"].lower()
        assert (await lc.add("default", "s", 1))[0] == 200
        code, b = await lc.add("default", "s", 2, entire=True)  # mounted → no entire
        assert code == 500
        assert (await lc.add("default", "s", 1))[0] == 200      # single after single: fine
    run(body)


def test_entire_mount_removes_as_a_whole():
    async def body(lc):
        lc.tenant("e")
        code, b = await lc.add("default", "e", 3, entire=True)
        assert code == 200 and len(b["devices"]) == 3
        assert len(lc.cluster.placeholders()) == 1             # one placeholder holds 3 GPUs
        ids = [d["bdf"] for d in b["devices"]]
        code, _ = await lc.remove("default", "e", ids[:2])     # partial removal refused
        assert code == 400
        code, b2 = await lc.remove("default", "e", ids)
        assert code == 200 and len(b2["devices"]) == 3
        assert lc.cluster.placeholders() == []
    run(body)


def test_single_mount_partial_removal_and_any_id_spelling():
    async def body(lc):
        lc.tenant("s")
        code, b = await lc.add("default", "s", 3)
        assert code == 200 and len(lc.cluster.placeholders()) == 3
        d0, d1 = b["devices"][0], b["devices"][1]
        code, _ = await lc.remove("default", "s", [d0["bdf"], "bogus"])
        assert code == 400 and len(lc.cluster.placeholders()) == 3  # nothing removed
        code, _ = await lc.remove("default", "s", [d0["uuid"], f"renderD{d1['render_minor']}"])
        assert code == 200 and len(lc.cluster.placeholders()) == 1
        assert not await lc.audit("default", "s")
        cid = lc.container_ids("default", "s")[0]
        devs = node_of(lc).container_devices(cid)
        assert "dev/kfd" in devs and len([d for d in devs if "renderD" in d]) == 1
    run(body)


def test_kfd_follows_first_and_last_gpu():
    async def body(lc):
        lc.tenant("k")
        cid = lc.container_ids("default", "k")[0]
        _, b1 = await lc.add("default", "k", 1)
        _, b2 = await lc.add("default", "k", 1)
        assert "dev/kfd" in node_of(lc).container_devices(cid)
        await lc.remove("default", "k", [b1["devices"][0]["uuid"]])
        assert "dev/kfd" in node_of(lc).container_devices(cid)
        await lc.remove("default", "k", [b2["devices"][0]["uuid"]])
        assert node_of(lc).container_devices(cid) == []
        assert not await lc.audit("default", "k")
    run(body)


# ------------------------------------------------------------------------------ busy / force
def test_busy_gpu_refused_then_force_kills(tmp_path, mock_inventory):
    sleeper = subprocess.Popen(["sleep", "60"])
    procs = tmp_path / "procs"
    _native.mock_smi().gm_mock_set_procs_file(str(procs).encode())
    try:
        async def body(lc):
            lc.tenant("busy", pids={"main": [sleeper.pid]})
            _, b = await lc.add("default", "busy", 1)
            dev = b["devices"][0]
            procs.write_text(f"{dev['index']} {sleeper.pid} 4096 python\n")
            code, text = await lc.remove("default", "busy", [dev["uuid"]], accept_json=False)
            assert (code, text) == (400, f"Pod: busy has running processes on GPU: "
                                         f"{dev['uuid']}\n")
            assert len(lc.cluster.placeholders()) == 1 and not await lc.audit("default", "busy")
            code, b2 = await lc.remove("default", "busy", [dev["uuid"]], force=True)
            assert code == 200 and b2["killed_pids"] == [sleeper.pid]
        # the busy process exists only in the mock amdsmi table (emulated device nodes are not
        # char devices an fd scan could see), so amdsmi must always be consulted
        run(body, worker_overrides={"busy_detection": "both"})
        sleeper.wait(timeout=10)
        assert sleeper.returncode == -15
    finally:
        _native.mock_smi().gm_mock_set_procs_file(b"")
        if sleeper.poll() is None:
            sleeper.kill()


def test_processes_outside_the_pod_do_not_make_it_busy(tmp_path, mock_inventory):
    procs = tmp_path / "procs"
    _native.mock_smi().gm_mock_set_procs_file(str(procs).encode())
    try:
        async def body(lc):
            lc.tenant("a", pids={"main": [os.getpid()]})
            _, b = await lc.add("default", "a", 1)
            procs.write_text(f"{b['devices'][0]['index']} 1 0 init\n")  # someone else's process
            code, _ = await lc.remove("default", "a", [b["devices"][0]["uuid"]])
            assert code == 200
        run(body, worker_overrides={"busy_detection": "both"})
    finally:
        _native.mock_smi().gm_mock_set_procs_file(b"")


# ------------------------------------------------------------------------------ variants
@pytest.mark.parametrize("cgroup_mode,driver,runtime", [
    ("v1", "cgroupfs", "docker"), ("v1", "systemd", "containerd"),
    ("v2", "systemd", "cri-o"), ("v2", "cgroupfs", "containerd")])
def test_runtime_and_cgroup_variants_with_multi_container_pods(cgroup_mode, driver, runtime):
    async def body(lc):
        lc.tenant("mc", containers=["trainer", "sidecar"], qos="burstable")
        code, b = await lc.add("default", "mc", 2)
        assert code == 200
        for cid in lc.container_ids("default", "mc"):
            devs = node_of(lc).container_devices(cid)
            assert sum("renderD" in d for d in devs) == 2 and "dev/kfd" in devs
        assert not await lc.audit("default", "mc")
        await lc.remove("default", "mc", [d["uuid"] for d in b["devices"]])
        for cid in lc.container_ids("default", "mc"):
            assert node_of(lc).container_devices(cid) == []
        assert not await lc.audit("default", "mc")
    run(body, cgroup_mode=cgroup_mode, cgroup_driver=driver, runtime=runtime)


def test_named_container_only():
    async def body(lc):
        lc.tenant("two", containers=["a", "b"])
        async with lc.session.get(lc.master_url + "/addgpu/namespace/default/pod/two/gpu/1/"
                                  "isEntireMount/false?container=b") as r:
            assert r.status == 200
        ca, cb = lc.container_ids("default", "two")
        assert node_of(lc).container_devices(ca) == []
        assert "dev/kfd" in node_of(lc).container_devices(cb)
    run(body)


def test_pod_with_own_gpus_keeps_them():
    """The pod's own device-plugin GPU is neither hot-managed nor removable, and does not make the
    pod look entire-mounted (reference defect 5)."""
    async def body(lc):
        lc.tenant("own", gpus=1)
        svc = lc.nodes["node-0"].worker.service
        st = await svc.pod_state(lc.cluster.get("default", "own"))
        assert len(st.own) == 1 and st.mount_type.value == "no-mount"
        assert (await lc.add("default", "own", 1))[0] == 200
        assert (await lc.add("default", "own", 1))[0] == 200   # still allowed
        code, _ = await lc.remove("default", "own", [st.own[0].uuid])
        assert code == 400                                     # own GPU is not removable
        cid = lc.container_ids("default", "own")[0]
        assert "dev/kfd" not in node_of(lc).container_devices(cid)  # runtime provides kfd
        assert not await lc.audit("default", "own")
    run(body)


# ------------------------------------------------------------------------------ topology
def test_scale_one_pod_1_to_8_then_0_in_xgmi_order():
    async def body(lc):
        lc.tenant("grow")
        got = []
        for _ in range(8):
            code, b = await lc.add("default", "grow", 1)
            assert code == 200
            got.append(b["devices"][0])
            assert not await lc.audit("default", "grow")
        assert [d["numa_node"] for d in got] == [0, 0, 0, 0, 1, 1, 1, 1]
        assert len({d["xgmi_hive_id"] for d in got}) == 1
        code, b = await lc.add("default", "grow", 1)
        assert code == 500 and "Insufficient" in b["message"]
        for d in reversed(got):
            assert (await lc.remove("default", "grow", [d["uuid"]]))[0] == 200
        assert lc.cluster.placeholders() == [] and not await lc.audit("default", "grow")
        assert node_of(lc).container_devices(lc.container_ids("default", "grow")[0]) == []
    run(body)


def test_placement_hint_followed_by_topology_plugin_and_counted_when_not():
    async def body(lc):
        lc.tenant("t")
        await lc.add("default", "t", 4, entire=True)
        m = lc.nodes["node-0"].worker.metrics
        assert m.placement_mismatch._value.get() == 0
    run(body)


def _numa_of(lc, devices):
    return {d["numa_node"] for d in devices}


def test_placement_hint_mode_with_stock_plugin_crosses_numa_and_is_counted():
    """hint only annotates: the stock plugin (first free in device order) never reads it."""
    async def body(lc):
        lc.tenant("other")
        lc.tenant("t")
        assert (await lc.add("default", "other", 3))[0] == 200      # first-free: GPUs 0,1,2
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        assert _numa_of(lc, b["devices"]) == {0, 1}                   # 3 and 4: across sockets
        assert lc.nodes["node-0"].worker.metrics.placement_mismatch._value.get() >= 1
    run(body, alloc_policy="first-free", worker_overrides={"placement_enforce": "hint"})


@pytest.mark.parametrize("entire", [False, True])
def test_default_placement_corrects_the_stock_plugins_choice(entire):
    """Default (auto) with a plugin that ignores the hint: the admitted set 3,4 crosses the
    socket, so the worker holds the other free GPUs, keeps two on NUMA 1 and releases the
    rest. The books end with exactly 3 + 2 GPUs."""
    async def body(lc):
        lc.tenant("other")
        lc.tenant("t")
        assert (await lc.add("default", "other", 3))[0] == 200
        code, b = await lc.add("default", "t", 2, entire=entire)
        assert code == 200, b
        assert _numa_of(lc, b["devices"]) == {1} and len(b["devices"]) == 2
        m = lc.nodes["node-0"].worker.metrics
        assert m.placement_corrections._value.get() == 1
        assert len(node_of(lc).allocated) == 5 and not await lc.audit("default", "t")
        code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
        assert code == 200 and len(node_of(lc).allocated) == 3
        # on an empty socket the plugin's own choice is already best: no correction round
        code, b2 = await lc.add("default", "t", 1)
        assert code == 200 and m.placement_corrections._value.get() == 1
    run(body, alloc_policy="first-free")


@pytest.mark.parametrize("entire", [False, True])
def test_placement_trim_enforces_topology_choice_with_blind_plugin(entire):
    async def body(lc):
        lc.tenant("other")
        lc.tenant("t")
        assert (await lc.add("default", "other", 3))[0] == 200
        code, b = await lc.add("default", "t", 2, entire=entire)
        assert code == 200
        assert _numa_of(lc, b["devices"]) == {1} and len(b["devices"]) == 2
        # surplus placeholders are gone; the books hold exactly 3 + 2 GPUs
        assert len(node_of(lc).allocated) == 5
        owners = sorted(p["metadata"]["labels"]["gpumounter.amd.com/owner"]
                        for p in lc.cluster.placeholders())
        assert owners == ["other"] * 3 + ["t"] * 2
        assert not await lc.audit("default", "t")
        if entire:   # the group removes as one entire mount
            code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
            assert code == 400                       # all-or-nothing (allocator.go:121-123)
            code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
            assert code == 200 and len(node_of(lc).allocated) == 3
        else:        # grow by one: stays on the same socket
            code, b2 = await lc.add("default", "t", 1)
            assert code == 200 and _numa_of(lc, b2["devices"]) == {1}
    run(body, alloc_policy="first-free", worker_overrides={"placement_enforce": "trim"})


# ------------------------------------------------------------------------------ namespaces/GC
def test_tenant_namespace_mode_garbage_collects_with_owner():
    async def body(lc):
        lc.tenant("t", ns="team-a")
        code, b = await lc.add("team-a", "t", 2)
        assert code == 200
        phs = lc.cluster.placeholders()
        assert {p["metadata"]["namespace"] for p in phs} == {"team-a"}
        assert all(p["metadata"]["ownerReferences"][0]["name"] == "t" for p in phs)
        lc.cluster.delete("team-a", "t", grace=0)
        await asyncio.sleep(0.05)
        assert lc.cluster.placeholders() == [] and node_of(lc).allocated == {}
    run(body, placeholder_namespace_mode="tenant")


def test_pool_mode_writes_no_cross_namespace_owner_refs():
    async def body(lc):
        lc.tenant("t")
        await lc.add("default", "t", 1)
        ph = lc.cluster.placeholders()[0]
        assert ph["metadata"]["namespace"] == "gpu-pool"
        assert "ownerReferences" not in ph["metadata"]
        assert lc.cluster.gc_sweep() == 0              # modern GC leaves it alone
        assert ph["metadata"]["labels"][LABEL_OWNER] == "t"
    run(body)


def test_owner_match_is_exact_not_substring():
    """Reference defect 3: pod 'a' saw the slaves of pod 'xa' (substring match)."""
    async def body(lc):
        lc.tenant("a")
        lc.tenant("xa")
        lc.tenant("a", ns="other")
        assert (await lc.add("default", "xa", 2))[0] == 200
        svc = lc.nodes["node-0"].worker.service
        for ns, name in (("default", "a"), ("other", "a")):
            st = await svc.pod_state(lc.cluster.get(ns, name))
            assert st.hot == [] and st.mount_type.value == "no-mount"
        assert (await lc.add("default", "a", 1, entire=True))[0] == 200
    run(body)


# ------------------------------------------------------------------------------ reconciler
def test_reconciler_collects_placeholders_of_deleted_owner():
    async def body(lc):
        lc.tenant("gone")
        await lc.add("default", "gone", 2)
        lc.cluster.delete("default", "gone", grace=0)
        rep = await lc.nodes["node-0"].worker.reconciler.run_once()
        assert len(rep.owner_gone) == 2
        await asyncio.sleep(0.05)
        assert lc.cluster.placeholders() == [] and node_of(lc).allocated == {}
    # the periodic sweep itself (the DELETED event would otherwise release them first)
    run(body, worker_overrides={"reconcile_on_events": False})


def test_reconciler_reinjects_after_container_restart():
    async def body(lc):
        lc.tenant("r")
        _, b = await lc.add("default", "r", 2)
        cid = lc.container_ids("default", "r")[0]
        ctr = node_of(lc).container(cid)
        # simulate a container restart: fresh /dev, fresh cgroup device state
        import shutil
        shutil.rmtree(os.path.join(ctr.root_dir, "dev"))
        os.makedirs(os.path.join(ctr.root_dir, "dev"))
        for f in ("devices.allow", "devices.deny"):
            open(os.path.join(ctr.cgroup_dir, f), "w").close()
        issues = await lc.audit("default", "r")
        assert {i.kind for i in issues} == {"missing_rule", "missing_node"}
        rep = await lc.nodes["node-0"].worker.reconciler.run_once()
        assert rep.repaired == ["default/r"]
        assert not await lc.audit("default", "r")
    run(body)


def test_reconciler_revokes_orphaned_state():
    async def body(lc):
        lc.tenant("o")
        _, b = await lc.add("default", "o", 1)
        # placeholder vanishes behind our back (e.g. deleted by an operator) → rules+nodes orphaned
        ph = lc.cluster.placeholders()[0]
        lc.cluster.delete(ph["metadata"]["namespace"], ph["metadata"]["name"], grace=0)
        await asyncio.sleep(0.05)
        issues = await lc.audit("default", "o")
        assert issues and all(i.kind.startswith("stale") for i in issues)
        rep = await lc.nodes["node-0"].worker.reconciler.run_once()
        assert rep.revoked == ["default/o"] and rep.orphans > 0
        assert not await lc.audit("default", "o")
    # the periodic sweep on its own (event-driven repair is covered further down)
    run(body, worker_overrides={"reconcile_on_events": False})


# ------------------------------------------------------------------------------ multi-node
def test_multi_node_routing_by_pod_node():
    async def body(lc):
        lc.tenant("n1pod", node="node-1")
        code, b = await lc.add("default", "n1pod", 2)
        assert code == 200
        phs = lc.cluster.placeholders()
        assert {p["spec"]["nodeName"] for p in phs} == {"node-1"}
        assert lc.nodes["node-0"].node.allocated == {}
        assert len(lc.nodes["node-1"].node.allocated) == 2
        svc1 = lc.nodes["node-1"].worker.service
        st = await svc1.pod_state(lc.cluster.get("default", "n1pod"))
        assert not svc1.hm.audit(lc.cluster.get("default", "n1pod"), st.hot, st.own)
    run(body, n_nodes=2)


def test_worker_restart_recovers_state_from_the_ledger():
    async def body(lc):
        lc.tenant("w")
        _, b = await lc.add("default", "w", 2)
        await lc.stop_worker("node-0")
        await lc.start_worker("node-0")
        await lc.master.workers.informer.wait_for(
            lambda: lc.master.workers.target("node-0") == f"127.0.0.1:"
            f"{lc.nodes['node-0'].worker.grpc_port}", 5)
        code, _ = await lc.remove("default", "w", [d["uuid"] for d in b["devices"]])
        assert code == 200 and not await lc.audit("default", "w")
    run(body)


# ------------------------------------------------------------------------------ observability
def test_status_endpoints_and_metrics():
    async def body(lc):
        lc.tenant("m")
        _, b = await lc.add("default", "m", 2)
        async with lc.session.get(lc.master_url + "/api/v1/nodes/node-0/gpus") as r:
            st = await r.json()
        assert len(st["gpus"]) == 8 and st["topology"]["all_pairs_xgmi"]
        assert sum(g["state"] == "GPU_ALLOCATED_STATE" for g in st["gpus"]) == 2
        async with lc.session.get(lc.master_url + "/api/v1/namespaces/default/pods/m/gpus") as r:
            mine = await r.json()
        assert len(mine["gpus"]) == 2
        w = lc.nodes["node-0"].worker
        async with lc.session.get(f"http://127.0.0.1:{w.http_port}/metrics") as r:
            text = await r.text()
        assert "gm_attach_latency_seconds_bucket" in text and 'stage="mount"' in text
        async with lc.session.get(f"http://127.0.0.1:{w.http_port}/readyz") as r:
            assert r.status == 200
        stages = {t["name"] for t in b["timings"]}
        assert {"ledger_reserve", "placeholder_wait", "mount", "mount.cgroup_rule",
                "mount.devnodes"} <= stages
    run(body)


def test_api_token_guards_mutating_routes():
    async def body(lc):
        lc.tenant("p")
        lc.master.cfg.api_token = "s3cret"
        code, text = await lc.add("default", "p", 1, accept_json=False)
        assert (code, text) == (401, "Unauthorized\n")
        url = lc.master_url + "/addgpu/namespace/default/pod/p/gpu/1/isEntireMount/false"
        async with lc.session.get(url, headers={"Authorization": "Bearer s3cret"}) as r:
            assert r.status == 200
        assert await text_get(lc, "/") == (200, "This is gpu mounter api!\n")  # read-only open
    run(body)


@pytest.mark.parametrize("index", [True, False])
def test_master_pod_cache_revalidates_recreated_and_deleted_pods(index):
    async def body(lc):
        lc.tenant("p", node="node-0")
        assert (await lc.add("default", "p", 1))[0] == 200          # fills the cache
        gets = lc.cluster.requests_by_verb.get("GET", 0)
        _, b = await lc.add("default", "p", 1)
        assert lc.cluster.requests_by_verb.get("GET", 0) == gets     # index hit: no GET
        # pod recreated on another node under the same name → worker refuses, master re-GETs
        lc.cluster.delete("default", "p", grace=0)
        lc.tenant("p", node="node-1")
        code, b = await lc.add("default", "p", 1)
        assert code == 200 and lc.cluster.placeholders()[-1]["spec"]["nodeName"] == "node-1"
        # pod deleted → reference semantics: 404 from the master, also for a request that
        # still finds the pod in the index (the watch has not delivered the deletion): the
        # worker's PodNotFound sends the master to a GET, which answers 404
        lc.cluster.delete("default", "p", grace=0)
        code, text = await lc.add("default", "p", 1, accept_json=False)
        assert (code, text) == (404, "No pod: p in namespace: default\n")
    run(body, n_nodes=2, master_overrides={"master_pod_index": index})


def test_idempotency_key_replays_instead_of_adding_more():
    async def body(lc):
        lc.tenant("i")
        url = lc.master_url + "/addgpu/namespace/default/pod/i/gpu/2/isEntireMount/false"
        hdr = {"Idempotency-Key": "job-42-attach", "Accept": "application/json"}
        async with lc.session.get(url, headers=hdr) as r:
            first = await r.json()
        async with lc.session.get(url, headers=hdr) as r:          # client retry
            again = await r.json()
        assert r.status == 200 and "replayed" in again["detail"]
        assert sorted(d["uuid"] for d in again["devices"]) == \
            sorted(d["uuid"] for d in first["devices"])
        assert len(lc.cluster.placeholders()) == 2                  # not 4
        assert not await lc.audit("default", "i")
    run(body)


def test_batch_endpoint_runs_operations_concurrently():
    async def body(lc):
        for t in ("b1", "b2", "b3"):
            lc.tenant(t)
        ops = {"operations": [{"op": "add", "pod": "b1", "gpus": 2},
                              {"op": "add", "pod": "b2", "gpus": 3, "entire": True},
                              {"op": "add", "pod": "b3", "gpus": 4},
                              {"op": "add", "pod": "ghost", "gpus": 1},
                              {"op": "frobnicate", "pod": "b1"}]}
        async with lc.session.post(lc.master_url + "/api/v1/batch", json=ops) as r:
            res = (await r.json())["results"]
        assert [x["code"] for x in res[:3]].count(200) >= 2     # 2+3+4 = 9 > 8: one must fail
        assert res[3]["code"] == 404 and res[4]["code"] == 400
        held = sum(len(x.get("devices", [])) for x in res[:3] if x["code"] == 200)
        assert held == len(lc.nodes["node-0"].node.allocated) <= 8
        rm = {"operations": [{"op": "remove", "pod": f"b{i + 1}",
                              "uuids": [d["uuid"] for d in x["devices"]]}
                             for i, x in enumerate(res[:3]) if x["code"] == 200]}
        async with lc.session.post(lc.master_url + "/api/v1/batch", json=rm) as r:
            assert all(x["code"] == 200 for x in (await r.json())["results"])
        assert lc.nodes["node-0"].node.allocated == {}
    run(body)


# ------------------------------------------------------------------------------ event-driven repair
async def _until(pred, timeout=3.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        if await pred():
            return True
        await asyncio.sleep(0.01)
    return False


def test_external_placeholder_delete_revokes_access_immediately():
    """kubectl delete / eviction of a placeholder returns its GPU to the scheduler: the tenant
    must lose access right away, not at the next periodic sweep (periodic reconcile is off)."""
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        victim = b["devices"][0]
        lc.cluster.delete(lc.cluster.placeholders()[0]["metadata"]["namespace"],
                          victim["placeholder"], grace=0)

        async def revoked():
            cid = lc.container_ids("default", "t")[0]
            return len(node_of(lc).container_devices(cid)) < 5 and \
                not await lc.audit("default", "t")
        assert await _until(revoked)
        st = await lc.nodes["node-0"].worker.service.pod_state(lc.cluster.get("default", "t"),
                                                               fresh=True)
        assert [g.bdf for g in st.hot] == [b["devices"][1]["bdf"]]
        assert lc.nodes["node-0"].worker.reconciler.event_actions >= 1
    run(body)


def test_tenant_delete_releases_placeholders_without_waiting_for_the_sweep():
    async def body(lc):
        lc.tenant("t")
        assert (await lc.add("default", "t", 3))[0] == 200
        lc.cluster.delete("default", "t", grace=0)

        async def released():
            return lc.cluster.placeholders() == [] and node_of(lc).allocated == {}
        assert await _until(released)
    run(body)


# ------------------------------------------------------------------------------ events / annotation
def test_attach_detach_emit_events_and_keep_devices_annotation():
    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        await svc.notify.drain()
        bdfs = sorted(d["bdf"] for d in b["devices"])
        ann = lc.cluster.get("default", "t")["metadata"]["annotations"]
        assert ann["gpumounter.amd.com/devices"] == ",".join(bdfs)
        code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
        assert code == 200
        await svc.notify.drain()
        ann = lc.cluster.get("default", "t")["metadata"]["annotations"]
        assert ann["gpumounter.amd.com/devices"] == b["devices"][1]["bdf"]
        lc.tenant("big")
        assert (await lc.add("default", "big", 8))[0] == 500        # 1 GPU held by t
        await svc.notify.drain()
        evs = lc.cluster.events_for("default", "t")
        assert [e["reason"] for e in evs] == ["GPUAttached", "GPUDetached"]
        assert all(e["involvedObject"]["uid"] == lc.cluster.get("default", "t")["metadata"]["uid"]
                   for e in evs)
        assert b["devices"][0]["bdf"] in evs[1]["message"]
        (fail,) = lc.cluster.events_for("default", "big")
        assert fail["reason"] == "GPUAttachFailed" and fail["type"] == "Warning"
        assert "gpumounter.amd.com/devices" not in (
            lc.cluster.get("default", "big")["metadata"].get("annotations") or {})
    run(body, worker_overrides={"annotate_tenant": True})


def test_external_delete_records_a_revocation_warning():
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 1)
        lc.cluster.delete(lc.cluster.placeholders()[0]["metadata"]["namespace"],
                          b["devices"][0]["placeholder"], grace=0)
        svc = lc.nodes["node-0"].worker.service

        async def warned():
            await svc.notify.drain()
            return any(e["reason"] == "GPURevoked" for e in lc.cluster.events_for("default", "t"))
        assert await _until(warned)
    run(body)


def test_notifications_wait_for_idle_worker_and_coalesce_annotations():
    """Events are never sent while an attach/detach is in flight; for one pod only the newest
    devices annotation is written (worker/notify.py)."""
    from types import SimpleNamespace

    from gpumounter_amd.worker.notify import Notifier

    class Kube:
        def __init__(self):
            self.calls = []

        async def create_event(self, ns, ev):
            self.calls.append(("event", ev["reason"]))

        async def patch_pod(self, ns, name, patch):
            self.calls.append(("patch", patch["metadata"]["annotations"]["gpumounter.amd.com/devices"]))

    async def body():
        cfg = SimpleNamespace(emit_events=True, annotate_tenant=True, node_name="n0",
                              notify_idle_ms=1.0, notify_max_delay_ms=10_000.0)
        kube = Kube()
        nt = Notifier(cfg, kube)
        pod = {"metadata": {"name": "t", "namespace": "default", "uid": "u1"}}
        g = lambda i: SimpleNamespace(index=i, bdf=f"0000:0{i}:00.0", render_minor=128 + i)  # noqa: E731
        with nt.operation():
            nt.attached(pod, [g(1)], [g(1)], "single")
            nt.attached(pod, [g(2)], [g(1), g(2)], "single")
            await asyncio.sleep(0.02)
            assert kube.calls == []                  # held back while the request runs
        await nt.drain()
        assert [c for c in kube.calls if c[0] == "event"] == [("event", "GPUAttached")] * 2
        assert [c for c in kube.calls if c[0] == "patch"] == [("patch", "0000:01:00.0,0000:02:00.0")]
        # under sustained load the max delay still flushes
        cfg.notify_max_delay_ms = 20.0
        kube.calls.clear()
        with nt.operation():
            nt.event(pod, "GPUDetached", "x")
            await asyncio.sleep(0.1)
            assert kube.calls == [("event", "GPUDetached")]
    asyncio.run(body())


def test_master_retries_unavailable_worker_and_the_retry_replays_not_duplicates():
    """AddGPU answered UNAVAILABLE (worker draining) is retried by the master's gRPC channel;
    the implicit idempotency key makes a retry of an attach that already happened a replay."""
    import grpc

    from gpumounter_amd.worker.service import RpcError

    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        real = svc.add_gpu
        calls = []

        async def flaky(req):
            calls.append(req.idempotency_key)
            if len(calls) == 1:
                await real(req)                  # the attach happens, the answer is lost
                raise RpcError(grpc.StatusCode.UNAVAILABLE, "worker draining")
            return await real(req)
        svc.add_gpu = flaky
        code, b = await lc.add("default", "t", 2)
        assert code == 200, b
        assert len(calls) == 2 and calls[0] == calls[1] != ""
        assert b["message"].startswith("Add GPU Success")
        st = await svc.pod_state(lc.cluster.get("default", "t"))
        assert len(st.hot) == 2                  # not 4
        assert await lc.audit("default", "t") == []
    run(body)


def test_tenant_deleted_mid_attach_reports_pod_not_found_and_leaks_nothing():
    from gpumounter_amd.fakes.apiserver import LatencyModel

    async def body(lc):
        lc.tenant("t")

        async def killer():
            await asyncio.sleep(0.015)            # while the placeholders are being admitted
            lc.cluster.delete("default", "t", grace=0)
        (code, b), _ = await asyncio.gather(lc.add("default", "t", 2), killer())
        assert code == 400 and b["add_gpu_result"] == "PodNotFound", b

        async def clean():
            live = [p for p in lc.cluster.placeholders()
                    if not p["metadata"].get("deletionTimestamp")]
            return not live and not node_of(lc).allocated
        assert await _until(clean)
    run(body, latency=LatencyModel(schedule_ms=30, admit_ms=20))


def test_remove_after_tenant_deleted_is_pod_not_found_and_releases():
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        lc.cluster.delete("default", "t", grace=0)
        code, r = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
        assert code in (400, 404), r          # master or worker: the pod is gone

        async def clean():
            live = [p for p in lc.cluster.placeholders()
                    if not p["metadata"].get("deletionTimestamp")]
            return not live and not node_of(lc).allocated
        assert await _until(clean)
    run(body)


def test_kubelet_restart_is_survived_without_waiting_for_grpc_backoff():
    """A kubelet restart recreates the PodResources socket; the ledger client rebuilds its
    channel on UNAVAILABLE, so the first attach after the restart already succeeds."""
    from gpumounter_amd.fakes.kubelet import FakeKubelet

    async def body(lc):
        lc.tenant("t")
        assert (await lc.add("default", "t", 1))[0] == 200
        h = lc.nodes["node-0"]
        await h.kubelet.stop()
        assert (await lc.add("default", "t", 1))[0] == 500        # kubelet down: refused
        h.kubelet = FakeKubelet(h.node, h.kubelet.socket_path)
        await h.kubelet.start()
        code, b = await lc.add("default", "t", 1)
        assert code == 200, b
        assert await lc.audit("default", "t") == []
    run(body, worker_overrides={"ledger_source": "podresources"})


def test_attach_reads_the_device_manager_checkpoint_not_the_podresources_socket():
    """ledger_source=auto (default): admission finds the placeholder's GPUs in the kubelet's
    device-manager checkpoint by pod UID — no PodResources call on the attach path, so an
    attach still works while that socket is down. A kubelet that does not maintain the
    checkpoint is detected (admitted placeholder, no entry) and PodResources takes over."""
    from gpumounter_amd.fakes.kubelet import FakeKubelet

    async def body(lc):
        lc.tenant("t")
        h = lc.nodes["node-0"]
        ph = h.worker.placeholders
        assert (await lc.add("default", "t", 1))[0] == 200   # first sight: one List (own GPUs)
        before = dict(h.kubelet.calls)
        code, b = await lc.add("default", "t", 2)
        assert code == 200, b
        assert h.kubelet.calls["Get"] == before["Get"] and \
            h.kubelet.calls["List"] == before["List"]
        assert ph.checkpoint_hits >= 1 and ph.checkpoint.trusted
        await h.kubelet.stop()
        assert (await lc.add("default", "t", 1))[0] == 200        # socket down: still served
        h.kubelet = FakeKubelet(h.node, h.kubelet.socket_path)
        await h.kubelet.start()
        assert await lc.audit("default", "t") == []
        # a kubelet without the checkpoint: three misses in a row, then PodResources only
        h.node.write_checkpoint = False
        os.unlink(h.node.checkpoint_path)
        for _ in range(3):
            code, b = await lc.add("default", "t", 1)
            assert code == 200, b
            code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
            assert code == 200
        assert h.kubelet.calls["Get"] >= 3
        h.node.write_checkpoint = True
        ckpt.write_atomic(h.node.checkpoint_path, ckpt.render([]))
        assert ph.checkpoint.lookup("anything") is None            # distrusted for good
        assert await lc.audit("default", "t") == []
    run(body)


def test_reconciler_sweep_makes_one_podresources_call_for_any_number_of_owners():
    """One authoritative List per sweep cross-checks the checkpoint; every owner is then
    audited from the checkpoint under its lock (the reference's pattern would be a kubelet
    dial per query: collector.go:90-138)."""
    async def body(lc):
        for i in range(4):
            lc.tenant(f"o{i}")
            assert (await lc.add("default", f"o{i}", 1))[0] == 200
        h = lc.nodes["node-0"]
        before = h.kubelet.calls["List"] + h.kubelet.calls["Get"]
        rep = await h.worker.reconciler.run_once()
        assert not rep.errors and not rep.repaired and not rep.revoked
        assert h.kubelet.calls["List"] + h.kubelet.calls["Get"] - before == 1
        assert h.worker.placeholders.checkpoint.trusted
    run(body)


def test_attach_verify_reads_back_rules_and_nodes_and_rolls_back_on_mismatch():
    """attach_verify: the attach reads its device rules and nodes back (span "verify"); when
    the kernel-side state does not match (here: the cgroup program reports nothing allowed),
    the attach fails and is rolled back instead of reporting success."""
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 1)
        assert code == 200, b
        assert "verify" in {t["name"] for t in b["timings"]}
        svc = lc.nodes["node-0"].worker.service
        real = svc.hm.backend.allowed
        svc.hm.backend.allowed = lambda cgdir: set()           # rules silently not in effect
        try:
            code, b2 = await lc.add("default", "t", 1)
        finally:
            svc.hm.backend.allowed = real
        assert code == 500 and "did not take effect" in str(b2), b2
        assert svc.metrics.verify_failures._value.get() == 1      # noqa: SLF001
        st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
        assert [g.uuid for g in st.hot] == [b["devices"][0]["uuid"]]   # only the first attach
        assert await lc.audit("default", "t") == []
        live = [p for p in lc.cluster.placeholders()
                if not p["metadata"].get("deletionTimestamp")]
        assert len(live) == 1
    run(body, worker_overrides={"attach_verify": True})


def test_shipped_default_places_optimally_on_a_fragmented_node_with_a_hint_blind_plugin():
    """with a device plugin that never reads the hint, the shipped
    default still yields one hive and NUMA-packed sets for N ≤ 4 whenever the free GPUs allow
    it (bench/configs.py placement; hint mode, for contrast, does not)."""
    import importlib.util
    import types

    spec = importlib.util.spec_from_file_location(
        "gm_configs", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench",
                                   "configs.py"))
    configs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(configs)
    args = types.SimpleNamespace(seed=3, rounds=25, sandbox=None)

    def scenario(mode):
        async def body(lc):
            return await configs.placement(lc, args)
        return run(body, alloc_policy="first-free",
                   worker_overrides={"placement_enforce": mode})
    auto = scenario("auto")
    for n, s in auto["per_n"].items():
        assert s["attaches"] > 0 and s["optimal"] == s["attaches"], (n, s)
        assert s["one_hive"] == s["attaches"] and s["numa_packed"] == s["numa_possible"], (n, s)
    assert auto["placement_corrections"] > 0 and auto["audit_issues"] == 0
    hint = scenario("hint")
    assert sum(s["optimal"] < s["attaches"] for s in hint["per_n"].values()) > 0, hint


def test_entire_mount_correction_takes_part_of_the_admitted_set_back():
    """Entire mount, best set = one GPU of the plugin's n-GPU placeholder + one other free GPU,
    and no n of the other free GPUs are as good: the placeholder is released and its GPUs taken
    back as 1-GPU placeholders (a second round), then the best pair is kept as a group."""
    async def body(lc):
        for t in ("a", "b", "t"):
            lc.tenant(t)
        gpus = lc.inventory.gpus()
        assert (await lc.add("default", "a", 3))[0] == 200               # 0,1,2 (NUMA 0)
        code, b = await lc.add("default", "b", 2)                        # a NUMA-1 pair
        assert code == 200 and _numa_of(lc, b["devices"]) == {1}
        held_b = {d["index"] for d in b["devices"]}
        free = [g.index for g in gpus if g.index not in held_b | {0, 1, 2}]
        code, c = await lc.add("default", "t", 2, entire=True)
        assert code == 200, c
        got = sorted(d["index"] for d in c["devices"])
        assert _numa_of(lc, c["devices"]) == {1}, (free, got)
        assert len(node_of(lc).allocated) == 7 and not await lc.audit("default", "t")
        code, _ = await lc.remove("default", "t", [c["devices"][0]["uuid"]])
        assert code == 400                                 # still one entire mount (group)
        code, _ = await lc.remove("default", "t", [d["uuid"] for d in c["devices"]])
        assert code == 200 and len(node_of(lc).allocated) == 5
    run(body, alloc_policy="first-free")


def test_entire_mount_correction_never_keeps_a_placeholder_it_let_go():
    """The second round of an entire-mount correction deletes the admitted placeholder, and that
    DELETE takes effect but its reply is lost. The attach must not fall back to "keeping the
    plugin's choice": that placeholder is gone, so its GPUs would be mounted with no booking
    and handed to the next Pod as well (found by chaos: one GPU attached to two Pods)."""
    from gpumounter_amd.cluster.placeholder import ReserveError

    async def body(lc):
        for t in ("a", "b", "t", "u"):
            lc.tenant(t)
        assert (await lc.add("default", "a", 3))[0] == 200
        assert (await lc.add("default", "b", 2))[0] == 200
        svc = lc.nodes["node-0"].worker.service
        real_release = svc.ph.release
        armed = {"on": True}

        async def release(phs, *a, **k):
            await real_release(phs, *a, **k)
            if armed["on"] and any(len(p.device_ids) > 1 for p in phs):
                armed["on"] = False
                raise ReserveError("DELETE applied, reply lost")
        svc.ph.release = release
        code, c = await lc.add("default", "t", 2, entire=True)
        assert not armed["on"], "the second round did not run"
        assert code != 200, c
        for _ in range(100):
            if len(node_of(lc).allocated) == 5:
                break
            await asyncio.sleep(0.02)
        assert len(node_of(lc).allocated) == 5               # only a's and b's GPUs booked
        assert not await lc.audit("default", "t")            # nothing left mounted in t
        code, d = await lc.add("default", "u", 3)            # every free GPU goes to u ...
        assert code == 200, d
        assert not await lc.audit("default", "u") and not await lc.audit("default", "t")
    run(body, alloc_policy="first-free")


def test_status_endpoints_answer_json_when_the_worker_is_down():
    async def body(lc):
        lc.tenant("m")
        target = lc.master.workers.target("node-0")
        await lc.stop_worker("node-0")
        lc.master.workers.target = lambda node: target      # the directory has not caught up
        async with lc.session.get(lc.master_url + "/api/v1/nodes/node-0/gpus") as r:
            assert r.status == 502 and "worker on node-0" in (await r.json())["error"]
        async with lc.session.get(lc.master_url + "/api/v1/namespaces/default/pods/m/gpus") as r:
            assert r.status == 502 and "UNAVAILABLE" in (await r.json())["error"]
    run(body)


def test_container_restart_gets_its_gpus_back_at_once():
    """A real restart: the runtime starts a new container (new id, cgroup and /dev). The worker
    reacts to the Pod's MODIFIED event — no periodic sweep involved — and puts the hot-mounted
    GPUs into the new container, with a GPUReinjected Event."""
    async def body(lc):
        lc.tenant("r")
        code, b = await lc.add("default", "r", 2)
        assert code == 200
        old = lc.container_ids("default", "r")[0]
        new = lc.cluster.restart_container("default", "r", "main")
        assert new != old and node_of(lc).container(old) is None
        w = lc.nodes["node-0"].worker
        for _ in range(100):
            await asyncio.sleep(0.02)
            if not await lc.audit("default", "r"):
                break
        assert not await lc.audit("default", "r")
        devs = node_of(lc).container_devices(new)
        assert sum("renderD" in d for d in devs) == 2 and "dev/kfd" in devs
        assert w.reconciler.event_actions >= 1
        for _ in range(100):        # Events are posted off the reaction's path
            reasons = [e["reason"] for e in lc.cluster.events_for("default", "r")]
            if "GPUReinjected" in reasons:
                break
            await asyncio.sleep(0.02)
        assert "GPUReinjected" in reasons
        code, _ = await lc.remove("default", "r", [d["uuid"] for d in b["devices"]])
        assert code == 200 and not node_of(lc).container_devices(new)
    run(body)          # LocalCluster runs no periodic sweep (reconcile_period_s=0)


def test_failed_event_reaction_is_retried_before_the_periodic_sweep():
    """A container restart's re-injection fails once (the kernel call is refused): the reaction
    is retried after a short backoff instead of waiting for the periodic sweep."""
    async def body(lc):
        lc.tenant("r")
        code, _ = await lc.add("default", "r", 1)
        assert code == 200
        w = lc.nodes["node-0"].worker
        hm = w.service.hm
        real, calls = hm.repair, []

        def flaky(*a, **k):
            calls.append(1)
            if len(calls) == 1:
                raise OSError("EBUSY: the kernel refused the program update")
            return real(*a, **k)
        hm.repair = flaky
        lc.cluster.restart_container("default", "r", "main")
        for _ in range(100):
            await asyncio.sleep(0.02)
            if not await lc.audit("default", "r"):
                break
        assert not await lc.audit("default", "r") and len(calls) == 2
        assert w.metrics.reconcile_actions.labels(action="event_retry")._value.get() == 1
    run(body)


def test_failed_attach_whose_cleanup_fails_is_followed_up_before_the_periodic_sweep():
    """An attach fails after its placeholder was admitted; releasing that placeholder fails
    (apiserver error) and so does the rollback's ledger read (the kubelet restarting). Both are
    handed to the reconciler's retrying follow-up: the placeholder is released and the Pod is
    left exactly as its ledger says within a second — LocalCluster runs no periodic sweep."""
    from gpumounter_amd.cluster.placeholder import ReserveError
    from gpumounter_amd.node.ledger import LedgerError

    async def body(lc):
        lc.tenant("f")
        w = lc.nodes["node-0"].worker
        svc = w.service
        real_release, real_by_pod = svc.ph.release, svc.ledger.by_pod
        calls = {"rel": 0, "led": -1}

        async def release(phs, *a, **k):
            calls["rel"] += 1
            if calls["rel"] == 1:
                calls["led"] = 0          # the rollback's ledger read fails next
                raise ReserveError("could not delete 1 placeholder(s): injected")
            return await real_release(phs, *a, **k)

        async def by_pod(*a, **k):
            if calls["led"] >= 0:
                calls["led"] += 1
            if calls["led"] == 1:
                raise LedgerError("kubelet PodResources socket unavailable")
            return await real_by_pod(*a, **k)
        svc.ph.release, svc.ledger.by_pod = release, by_pod
        def held():
            return [p for p in lc.cluster.placeholders() if (p["metadata"].get("annotations")
                    or {}).get("gpumounter.amd.com/owner-name") == "f"]
        code, _ = await lc.add("default", "f", 1)
        assert code == 500
        for _ in range(250):           # retries at 0.1, 0.5 s: a loaded host needs longer
            await asyncio.sleep(0.02)
            if not held() and not await lc.audit("default", "f"):
                break
        assert not held()
        assert not await lc.audit("default", "f")
        assert not node_of(lc).container_devices(lc.container_ids("default", "f")[0])
        assert calls["rel"] >= 2 and calls["led"] >= 2
        assert w.metrics.reconcile_actions.labels(action="followup_release")._value.get() == 1
    run(body, worker_overrides={"fault": "devnodes:1.0:after"})


def test_sweep_that_hit_errors_runs_again_before_the_next_period():
    """A sweep that could not finish (here: its ledger read failed) is repeated after a short
    backoff, not a whole period (30 s as shipped) later; a clean one waits the period."""
    from gpumounter_amd.worker.reconciler import ReconcileReport, Reconciler

    async def main():
        r = Reconciler(service=None, period_s=30.0)
        reports = [ReconcileReport(errors=["ledger: kubelet restarting"]), ReconcileReport()]
        calls = []

        async def run_once():
            calls.append(asyncio.get_running_loop().time())
            return reports[min(len(calls), len(reports)) - 1]
        r.run_once = run_once
        await r.start()
        await asyncio.sleep(1.0)
        await r.stop()
        assert len(calls) == 2                       # at once, again after 0.5 s, then 30 s
        assert 0.4 < calls[1] - calls[0] < 0.9
    asyncio.run(main())


def test_container_restart_during_an_attach_gets_the_gpus():
    """The tenant's container restarts while its first attach is reserving: the Pod event comes
    before the placeholder exists, so the event-driven re-injection does not see a Pod with
    hot-mounted GPUs. The attach mounts the container running now, not the one it looked up
    (no periodic sweep here)."""
    async def body(lc):
        lc.tenant("c")
        svc = lc.nodes["node-0"].worker.service
        real = svc.ph.reserve
        restarted = []

        async def reserve(*a, **k):
            res = await real(*a, **k)
            if not restarted:
                restarted.append(lc.cluster.restart_container("default", "c", "main"))
                await asyncio.sleep(0.05)        # the Pod event is delivered meanwhile
            return res
        svc.ph.reserve = reserve
        code, b = await lc.add("default", "c", 1)
        svc.ph.reserve = real
        assert code == 200 and restarted
        assert lc.container_ids("default", "c") == restarted
        assert not await lc.audit("default", "c")
        devs = node_of(lc).container_devices(restarted[0])
        assert sum("renderD" in d for d in devs) == 1 and "dev/kfd" in devs
    run(body)


def test_container_restart_between_mount_and_read_back_rolls_the_attach_back():
    """The container restarts between the mount and its read-back (the control plane runs in
    another process, so this interleaving is real): the read-back fails on the vanished
    container, and the attach is rolled back — placeholder released, nothing in the new
    container — instead of escaping unhandled with its placeholder left behind."""
    async def body(lc):
        lc.tenant("v")
        svc = lc.nodes["node-0"].worker.service
        real_attach = svc.hm.attach

        def attach(*a, **k):
            out = real_attach(*a, **k)
            lc.cluster.restart_container("default", "v", "main")
            return out
        svc.hm.attach = attach
        code, _ = await lc.add("default", "v", 1)
        svc.hm.attach = real_attach
        assert code == 500
        assert not [p for p in lc.cluster.placeholders()
                    if (p["metadata"].get("annotations") or {}).get(
                        "gpumounter.amd.com/owner-name") == "v"]
        assert not await lc.audit("default", "v")
        assert not node_of(lc).container_devices(lc.container_ids("default", "v")[0])
        code, _ = await lc.add("default", "v", 1)       # and the next attach works
        assert code == 200 and not await lc.audit("default", "v")
    run(body)


def test_relist_wakes_the_sweep():
    """A watch that relisted (410 Gone, a dropped stream) missed events, which no reaction saw:
    the relist wakes the sweep instead of leaving their effects to the next period (30 s)."""
    from gpumounter_amd.worker.reconciler import ReconcileReport, Reconciler

    async def main():
        r = Reconciler(service=None, period_s=30.0)
        calls = []

        async def run_once():
            calls.append(asyncio.get_running_loop().time())
            return ReconcileReport()
        r.run_once = run_once
        r.WAKE_MIN_INTERVAL_S = 0.2
        await r.start()
        await asyncio.sleep(0.05)
        r._on_node_pod("RELIST", {})
        await asyncio.sleep(0.05)
        r._on_relist("RELIST", {})      # before the woken sweep started: that sweep covers it
        r._on_relist("MODIFIED", {})    # not a relist
        await asyncio.sleep(0.3)
        assert len(calls) == 2 and calls[1] - calls[0] >= 0.19   # at most 1 per 0.2 s
        r._on_relist("RELIST", {})      # the placeholder informer
        await asyncio.sleep(0.3)
        await r.stop()
        assert len(calls) == 3 and r.woken == 2
    asyncio.run(main())


def test_sweep_loop_survives_a_cancelled_inner_await():
    """Something the sweep awaited was cancelled under it (a CancelledError that stop() did
    not cause): that sweep failed, the loop goes on and retries after a short backoff. Only
    stop() ends it."""
    from gpumounter_amd.worker.reconciler import ReconcileReport, Reconciler

    async def main():
        r = Reconciler(service=None, period_s=30.0)
        calls = []

        async def run_once():
            calls.append(1)
            if len(calls) == 1:
                raise asyncio.CancelledError()
            return ReconcileReport()
        r.run_once = run_once
        await r.start()
        await asyncio.sleep(0.8)
        assert len(calls) == 2 and not r._task.done()
        await r.stop()
        assert r._task.done()
    asyncio.run(main())


def test_retry_under_the_key_of_a_failed_attach_does_not_replay_its_leftover():
    """An attach fails and its placeholder cannot be released yet (the follow-up keeps
    retrying). The client retries under the same Idempotency-Key: the leftover must not be
    replayed as that request's success — the client was told it failed, and the follow-up is
    about to release it. The retry attaches afresh."""
    from gpumounter_amd.cluster.placeholder import ReserveError

    async def body(lc):
        lc.tenant("k")
        w = lc.nodes["node-0"].worker
        svc = w.service
        real_release = svc.ph.release
        fail = {"on": True}

        async def release(phs, *a, **k):
            if fail["on"]:
                raise ReserveError("could not delete placeholder(s): apiserver unavailable")
            return await real_release(phs, *a, **k)
        svc.ph.release = release
        url = f"{lc.master_url}/addgpu/namespace/default/pod/k/gpu/1/isEntireMount/false"
        hdr = {"Accept": "application/json", "Idempotency-Key": "req-1"}
        async with lc.session.get(url, headers=hdr) as r:
            assert r.status == 500
        left = [p for p in lc.cluster.placeholders()
                if (p["metadata"].get("annotations") or {}).get(
                    "gpumounter.amd.com/owner-name") == "k"]
        assert len(left) == 1 and left[0]["metadata"]["uid"] in svc.abandoned
        svc.hm.faults.rules.pop("devnodes")
        async with lc.session.get(url, headers=hdr) as r:
            assert r.status == 200
            b = await r.json()
        assert "replayed" not in b.get("message", "")
        assert [d["placeholder"] for d in b["devices"]] != [left[0]["metadata"]["name"]]
        # neither the rollback nor the retry mounted the leftover's GPU: once the follow-up
        # deletes it the scheduler may hand it out, so the tenant must never have reached it
        assert not await lc.audit("default", "k")
        fail["on"] = False                   # the apiserver is back: the follow-up drops it
        for _ in range(150):
            await asyncio.sleep(0.02)
            if not svc.abandoned:
                break
        assert not svc.abandoned
        names = {p["metadata"]["name"] for p in lc.cluster.placeholders()}
        assert left[0]["metadata"]["name"] not in names
        assert not await lc.audit("default", "k")
    run(body, worker_overrides={"fault": "devnodes:1.0:after"})


def test_candidates_of_a_failed_trim_pick_are_released_by_the_follow_up():
    """A trim pick holds every free GPU as candidates; confirming the kept ones fails, and so
    does the pick's own cleanup (apiserver errors). The leftover candidates hold GPUs nobody
    uses: the follow-up releases them at once instead of the next periodic sweep (none runs
    here)."""
    from gpumounter_amd.cluster.placeholder import ReserveError

    async def body(lc):
        lc.tenant("tp")
        svc = lc.nodes["node-0"].worker.service
        real_confirm, real_release = svc.ph.confirm, svc.ph.release
        calls = {"confirm": 0, "release": 0}

        async def confirm(phs):
            calls["confirm"] += 1
            if calls["confirm"] == 1:
                raise ReserveError("confirming 1 placeholder(s) failed: 503")
            return await real_confirm(phs)

        async def release(phs, *a, **k):
            calls["release"] += 1
            if calls["release"] == 1:
                raise ReserveError("could not delete 8 placeholder(s): 503")
            return await real_release(phs, *a, **k)
        svc.ph.confirm, svc.ph.release = confirm, release
        code, _ = await lc.add("default", "tp", 1)
        assert code == 500 and calls["release"] >= 1
        for _ in range(100):
            await asyncio.sleep(0.02)
            if not lc.cluster.placeholders():
                break
        assert lc.cluster.placeholders() == []
        assert not lc.nodes["node-0"].node.allocated
        assert not await lc.audit("default", "tp")
        code, _ = await lc.add("default", "tp", 1)          # and the node is usable again
        assert code == 200
    run(body, alloc_policy="first-free", worker_overrides={"placement_enforce": "trim"})


def test_placement_correct_on_xgmi_leaves_numa_only_differences_alone():
    """placement_correct_on=xgmi: on a node whose GPUs all share one hive (the mock MI355X
    node), a plugin pick that only crosses the socket is kept — no correction round, no
    exclusive hold of every free GPU (the cost of the default)."""
    async def body(lc):
        lc.tenant("other")
        lc.tenant("t")
        assert (await lc.add("default", "other", 3))[0] == 200
        code, b = await lc.add("default", "t", 2)
        assert code == 200 and _numa_of(lc, b["devices"]) == {0, 1}, b
        assert lc.nodes["node-0"].worker.metrics.placement_corrections._value.get() == 0
        assert len(node_of(lc).allocated) == 5 and not await lc.audit("default", "t")
    run(body, alloc_policy="first-free", worker_overrides={"placement_correct_on": "xgmi"})


def test_identical_queued_events_are_sent_once_with_their_count():
    """A Pod attached and detached in a loop while notifications are held back: the flush sends
    one Event per (Pod, reason, message) with its count — client-go's aggregation — instead of
    a burst of one request per operation on the worker's event loop."""
    from types import SimpleNamespace

    from gpumounter_amd.worker.notify import Notifier

    class Kube:
        def __init__(self):
            self.events = []

        async def create_event(self, ns, ev):
            self.events.append(dict(ev))

    async def body():
        cfg = SimpleNamespace(emit_events=True, annotate_tenant=False, node_name="n0",
                              notify_idle_ms=1.0, notify_max_delay_ms=10_000.0)
        kube = Kube()
        nt = Notifier(cfg, kube)
        pod = {"metadata": {"name": "t", "namespace": "default", "uid": "u1"}}
        g = SimpleNamespace(index=1, bdf="0000:01:00.0", render_minor=129)
        with nt.operation():
            for _ in range(50):
                nt.attached(pod, [g], [g], "entire")
                nt.detached(pod, [g], [], [])
            nt.attached(pod, [g], [g], "single")          # another message: its own Event
        await nt.drain()
        got = sorted((e["reason"], e["count"], e["message"][:20]) for e in kube.events)
        assert got == [("GPUAttached", 1, "hot-mounted 1 GPU(s)"),
                       ("GPUAttached", 50, "hot-mounted 1 GPU(s)"),
                       ("GPUDetached", 50, "removed 1 GPU(s): 00")], got
        # after the flush a new one starts a new aggregate
        with nt.operation():
            nt.detached(pod, [g], [], [])
        await nt.drain()
        assert kube.events[-1]["count"] == 1
    asyncio.run(body())


def test_master_opens_worker_channels_before_the_first_request():
    """The master connects to every running worker it discovers (TCP, and TLS where set), so
    the first attach does not pay the handshake."""
    import grpc

    async def main():
        async with LocalCluster() as lc:
            wd = lc.master.workers
            target = wd.target("node-0")
            assert target is not None
            state = None
            for _ in range(250):
                ch = wd._channels.get(target)                       # noqa: SLF001
                state = ch.get_state() if ch is not None else None
                if state == grpc.ChannelConnectivity.READY:
                    break
                await asyncio.sleep(0.02)
            assert state == grpc.ChannelConnectivity.READY
    asyncio.run(main())
