"""amd.com/gpu device plugin (gpumounter_amd/deviceplugin) against the fake kubelet's device
manager: registration, ListAndWatch health, Allocate device specs, GetPreferredAllocation
steering, kubelet restart."""
import asyncio
import os

import grpc

from gpumounter_amd.api import deviceplugin as dp
from gpumounter_amd.fakes.harness import LocalCluster


def run(body, **kw):
    async def main():
        async with LocalCluster(device_plugin=True, **kw) as lc:
            return await body(lc)
    return asyncio.run(main())


def test_schema_wire_bytes():
    r = dp.ContainerAllocateResponse(envs={"A": "1"})
    r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    assert r.SerializeToString().hex() == \
        "0a060a01411201311a180a082f6465762f6b666412082f6465762f6b66641a027277"
    req = dp.RegisterRequest(version="v1beta1", endpoint="x.sock", resource_name="amd.com/gpu",
                             options=dp.DevicePluginOptions(get_preferred_allocation_available=True))
    assert req.SerializeToString() == b'\n\x07v1beta1\x12\x06x.sock\x1a\x0bamd.com/gpu"\x02\x10\x01'


def test_registers_and_advertises_inventory_with_numa():
    async def body(lc):
        h = lc.nodes["node-0"]
        assert h.kubelet.calls["Register"] == 1 and h.node.plugin is h.kubelet
        devs = h.kubelet.plugin_devices
        assert len(devs) == 8 and set(devs.values()) == {dp.HEALTHY}
        assert sorted(devs) == sorted(g.bdf for g in h.node.gpus)
    run(body)


def test_allocate_returns_kfd_render_and_card_specs():
    async def body(lc):
        plugin = lc.nodes["node-0"].worker.plugin
        async with grpc.aio.insecure_channel(f"unix://{plugin.socket_path}") as ch:
            alloc = ch.unary_unary(dp.ALLOCATE, dp.AllocateRequest.SerializeToString,
                                   dp.AllocateResponse.FromString)
            req = dp.AllocateRequest()
            req.container_requests.add(devices_ids=["0000:15:00.0"])
            resp = await alloc(req)
            paths = [d.container_path for d in resp.container_responses[0].devices]
            assert paths == ["/dev/kfd", "/dev/dri/renderD129", "/dev/dri/card1"]
            req = dp.AllocateRequest()
            req.container_requests.add(devices_ids=["0000:ff:00.0"])
            try:
                await alloc(req)
                raise AssertionError("unknown device accepted")
            except grpc.aio.AioRpcError as e:
                assert e.code() == grpc.StatusCode.INVALID_ARGUMENT
    run(body)


def test_unhealthy_device_is_not_allocated():
    async def body(lc):
        h = lc.nodes["node-0"]
        h.worker.plugin.set_health(0, False)
        for _ in range(100):
            if h.kubelet.plugin_devices.get(h.node.gpus[0].bdf) == dp.UNHEALTHY:
                break
            await asyncio.sleep(0.01)
        assert h.node.gpus[0].bdf in h.node.unhealthy
        lc.tenant("t")
        code, b = await lc.add("default", "t", 7)
        assert code == 200 and h.node.gpus[0].bdf not in {d["bdf"] for d in b["devices"]}
        lc.tenant("u")
        code, _ = await lc.add("default", "u", 1)
        assert code == 500                       # the only free GPU is unhealthy
    run(body)


def test_preferred_allocation_steers_to_the_workers_choice():
    """Growing a pod: the worker's choice is NUMA-aware relative to the pod's GPUs, which the
    plugin alone (no pod identity in GetPreferredAllocation) cannot know."""
    async def body(lc):
        h = lc.nodes["node-0"]
        lc.tenant("other")
        lc.tenant("t")
        code, bo = await lc.add("default", "other", 4)           # NUMA 0 filled
        assert code == 200 and {d["numa_node"] for d in bo["devices"]} == {0}
        code, b1 = await lc.add("default", "t", 1)
        assert code == 200 and b1["devices"][0]["numa_node"] == 1
        assert (await lc.remove("default", "other", [d["uuid"] for d in bo["devices"]]))[0] == 200
        before = h.worker.plugin.calls["steered"]
        code, b2 = await lc.add("default", "t", 1)
        assert code == 200 and b2["devices"][0]["numa_node"] == 1
        assert h.worker.plugin.calls["steered"] > before
        assert h.worker.metrics.placement_mismatch._value.get() == 0
        assert not h.worker.plugin.intents                       # consumed or withdrawn
        assert not await lc.audit("default", "t")
    run(body)


def test_plugin_reregisters_after_kubelet_restart():
    async def body(lc):
        h = lc.nodes["node-0"]
        await h.kubelet.restart()
        assert h.node.plugin is None
        for _ in range(400):
            if h.node.plugin is not None:
                break
            await asyncio.sleep(0.01)
        assert h.kubelet.calls["Register"] == 2 and os.path.exists(h.worker.plugin.socket_path)
        lc.tenant("t")
        assert (await lc.add("default", "t", 2))[0] == 200
    run(body)


def test_standalone_device_plugin_cli_serves_the_api(tmp_path):
    """python -m gpumounter_amd device-plugin: the plugin without a worker."""
    import subprocess
    import sys

    d = tmp_path / "dp"
    d.mkdir()
    proc = subprocess.Popen([sys.executable, "-m", "gpumounter_amd", "device-plugin",
                             "--amdsmi", "mock", "--dir", str(d), "--no-register"],
                            stdout=subprocess.PIPE, text=True,
                            env={**os.environ, "GM_LOG_JSON": "0"})
    try:
        line = proc.stdout.readline()
        info = __import__("json").loads(line)
        assert info["devices"] == 8

        async def call():
            async with grpc.aio.insecure_channel(f"unix://{info['socket']}") as ch:
                law = ch.unary_stream(dp.LIST_AND_WATCH, dp.Empty.SerializeToString,
                                      dp.ListAndWatchResponse.FromString)
                async for resp in law(dp.Empty()):
                    return resp
        resp = asyncio.run(call())
        assert len(resp.devices) == 8 and all(x.health == dp.HEALTHY for x in resp.devices)
        assert {x.topology.nodes[0].ID for x in resp.devices} == {0, 1}
    finally:
        proc.terminate()
        assert proc.wait(timeout=20) == 0


def test_worker_exports_device_plugin_metrics():
    async def body(lc):
        lc.tenant("t")
        assert (await lc.add("default", "t", 2))[0] == 200
        w = lc.nodes["node-0"].worker
        await w.collect_metrics()
        text = w.metrics.render().decode()
        assert 'gm_device_plugin_rpcs_total{rpc="Allocate"} 2.0' in text
        assert "gm_device_plugin_healthy_gpus 8.0" in text
    run(body)


def test_new_uncorrectable_ecc_error_takes_a_gpu_out_of_service():
    """ecc_policy=new: a GPU whose uncorrectable ECC count rises is reported Unhealthy to the
    kubelet (so no placeholder can get it), left out of placement, flagged in /status and in
    gm_gpu_healthy; pre-existing errors at worker start do not count."""
    import asyncio

    from gpumounter_amd import _native
    from gpumounter_amd.fakes.harness import LocalCluster

    mock = _native.mock_smi()

    async def main():
        mock.gm_mock_set_ecc(3, 5, 2)            # errors on record before the worker starts
        try:
            async with LocalCluster(device_plugin=True,
                                    worker_overrides={"health_period_s": 0}) as lc:
                w = lc.nodes["node-0"].worker
                await w.check_health()
                assert w.service.unhealthy == set()          # policy "new": history is fine
                mock.gm_mock_set_ecc(0, 0, 1)                # a fresh uncorrectable error
                await w.check_health()
                assert w.service.unhealthy == {0}
                bad_bdf = next(g.bdf for g in lc.inventory.gpus() if g.index == 0)
                text = w.metrics.render().decode()
                assert f'gm_gpu_healthy{{gpu="{bad_bdf}"}} 0.0' in text

                async def plugin_saw_it():
                    return bool(lc.nodes["node-0"].node.unhealthy)
                for _ in range(100):
                    if await plugin_saw_it():
                        break
                    await asyncio.sleep(0.02)
                assert await plugin_saw_it()
                lc.tenant("t")
                code, b = await lc.add("default", "t", 7)
                assert code == 200, b
                assert bad_bdf not in {d["bdf"] for d in b["devices"]}
                lc.tenant("u")
                assert (await lc.add("default", "u", 1))[0] == 500   # only the sick GPU is left
                st = await w.service.node_status(False)
                assert [g["healthy"] for g in st["gpus"] if g["index"] == 0] == [False]
        finally:
            mock.gm_mock_set_ecc(0, 0, 0)
            mock.gm_mock_set_ecc(3, 0, 0)
    asyncio.run(main())
