"""The kubelet device-manager checkpoint reader (gpumounter_amd/node/checkpoint.py)."""
import asyncio
import json
import os

import pytest

from gpumounter_amd.node import checkpoint as ckpt

V2 = {"Data": {"PodDeviceEntries": [
    {"PodUID": "u1", "ContainerName": "a", "ResourceName": "amd.com/gpu",
     "DeviceIDs": {"1": ["0000:85:00.0"], "0": ["0000:05:00.0"]}, "AllocResp": "Cg=="},
    {"PodUID": "u1", "ContainerName": "b", "ResourceName": "amd.com/gpu",
     "DeviceIDs": {"0": ["0000:15:00.0"]}, "AllocResp": ""},
    {"PodUID": "u2", "ContainerName": "a", "ResourceName": "example.com/nic",
     "DeviceIDs": {"0": ["nic0"]}, "AllocResp": ""}],
    "RegisteredDevices": {"amd.com/gpu": ["0000:05:00.0"]}}, "Checksum": 42}


def test_parse_v2_groups_by_uid_numa_ordered_and_filters_resource():
    got = ckpt.parse(json.dumps(V2).encode(), "amd.com/gpu")
    assert got == {"u1": ("0000:05:00.0", "0000:85:00.0", "0000:15:00.0")}


def test_parse_pre_1_20_flat_list_and_empty():
    doc = {"Data": {"PodDeviceEntries": [{"PodUID": "u", "ContainerName": "c",
                                          "ResourceName": "amd.com/gpu",
                                          "DeviceIDs": ["renderD128"], "AllocResp": ""}],
                    "RegisteredDevices": {}}, "Checksum": 1}
    assert ckpt.parse(json.dumps(doc).encode(), "amd.com/gpu") == {"u": ("renderD128",)}
    empty = {"Data": {"PodDeviceEntries": None, "RegisteredDevices": None}, "Checksum": 0}
    assert ckpt.parse(json.dumps(empty).encode(), "amd.com/gpu") == {}


@pytest.mark.parametrize("blob", [b"", b"{", b"[]", b'{"Data": 3}',
                                  b'{"Data": {"PodDeviceEntries": [1]}}',
                                  b'{"Data": {"PodDeviceEntries": [{"PodUID": "u", '
                                  b'"ResourceName": "amd.com/gpu", "DeviceIDs": 7}]}}'])
def test_parse_rejects_what_is_not_a_checkpoint(blob):
    with pytest.raises(ckpt.CheckpointFormatError):
        ckpt.parse(blob, "amd.com/gpu")


def test_render_round_trips():
    blob = ckpt.render([("u9", "main", "amd.com/gpu", {0: ["a", "b"], 1: ["c"]})],
                       {"amd.com/gpu": ["a", "b", "c"]})
    assert ckpt.parse(blob, "amd.com/gpu") == {"u9": ("a", "b", "c")}


def test_reader_parses_only_when_the_file_changes(tmp_path):
    path = str(tmp_path / ckpt.CHECKPOINT_NAME)
    r = ckpt.DeviceCheckpoint(path, "amd.com/gpu")
    assert r.snapshot() is None and r.lookup("u1") is None      # absent
    ckpt.write_atomic(path, json.dumps(V2).encode())
    assert r.lookup("u1")[0] == "0000:05:00.0" and r.parses == 1
    for _ in range(5):
        assert r.lookup("u2") is None
    assert r.parses == 1                                        # no re-parse while unchanged
    ckpt.write_atomic(path, ckpt.render([("u2", "c", "amd.com/gpu", {0: ["x"]})]))
    assert r.lookup("u2") == ("x",) and r.lookup("u1") is None and r.parses == 2
    with open(path, "wb") as fh:
        fh.write(b"garbage")
    assert r.snapshot() is None and r.errors == 1
    r.distrust("test")
    ckpt.write_atomic(path, json.dumps(V2).encode())
    assert r.lookup("u1") is None                               # distrusted for good


def test_inotify_wakes_on_the_kubelets_rename(tmp_path):
    path = str(tmp_path / ckpt.CHECKPOINT_NAME)

    async def body():
        r = ckpt.DeviceCheckpoint(path, "amd.com/gpu")
        woke = asyncio.Event()
        assert r.watch(woke.set)
        try:
            with open(tmp_path / "unrelated", "w") as fh:   # other files do not wake
                fh.write("x")
            await asyncio.sleep(0.05)
            assert not woke.is_set()
            ckpt.write_atomic(path, ckpt.render([("u", "c", "amd.com/gpu", {0: ["g"]})]))
            await asyncio.wait_for(woke.wait(), 2)
            return r.lookup("u")
        finally:
            r.close()
    assert asyncio.run(body()) == ("g",)
    assert not ckpt.DeviceCheckpoint(str(tmp_path / "nodir" / "x"), "r").watch(lambda: None)
    assert os.path.exists(path)


def test_cross_check_distrusts_after_consecutive_disagreements(tmp_path):
    path = str(tmp_path / ckpt.CHECKPOINT_NAME)
    ckpt.write_atomic(path, ckpt.render([("u1", "c", "amd.com/gpu", {0: ["a"]})]))
    r = ckpt.DeviceCheckpoint(path, "amd.com/gpu")
    uids = {("ns", "p1"): "u1", ("ns", "p2"): "u2"}
    assert r.cross_check({("ns", "p1"): ["a"]}, uids.get)
    assert r.cross_check({("ns", "p1"): ["a"], ("ns", "x"): ["b"]}, uids.get)  # unknown uid
    assert r.by_name([{"metadata": {"namespace": "ns", "name": "p1", "uid": "u1"}},
                      {"metadata": {"namespace": "ns", "name": "p2", "uid": "u2"}}]) == \
        {("ns", "p1"): ["a"]}
    assert not r.cross_check({("ns", "p2"): ["b"]}, uids.get)                  # 1st miss
    assert r.cross_check({("ns", "p1"): ["a"]}, uids.get) and r.mismatches == 0  # reset
    for _ in range(3):
        assert not r.cross_check({("ns", "p1"): ["z"]}, uids.get)
    assert not r.trusted and r.by_name([]) is None and r.lookup("u1") is None


def test_same_size_rewrite_in_the_same_tick_is_seen(tmp_path):
    """The kubelet's tmp + rename reuses the inode just freed and two rewrites inside one
    timestamp tick share an mtime: a swap of one UID for another of the same length must still
    be seen (stat metadata cannot key the cache)."""
    path = str(tmp_path / ckpt.CHECKPOINT_NAME)
    r = ckpt.DeviceCheckpoint(path, "amd.com/gpu")
    ckpt.write_atomic(path, ckpt.render([("uid-a", "c", "amd.com/gpu", {0: ["g0"]})]))
    st = os.stat(path)
    assert r.lookup("uid-a") == ("g0",)
    ckpt.write_atomic(path, ckpt.render([("uid-b", "c", "amd.com/gpu", {0: ["g0"]})]))
    os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns))        # same tick
    assert os.stat(path).st_size == st.st_size
    assert r.lookup("uid-b") == ("g0",) and r.lookup("uid-a") is None


def test_ledger_reporting_more_devices_than_requested_fails_the_attach():
    """A placeholder requesting 1 GPU for which the kubelet ledger reports 2 (a kubelet or
    device-plugin inconsistency): mounting both would give the tenant a GPU the scheduler
    still counts as free, so the attach fails, is rolled back, and its placeholder released."""
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.fakes.node import FakeNode

    orig = FakeNode.allocate

    def over_allocate(self, ns, pod, container, n, uid=""):
        ids = orig(self, ns, pod, container, n, uid)
        if ids and "-slave-pod-" in pod:
            extra = orig(self, ns, pod, container, 1, uid)   # a second Allocate
            ids = ids + (extra or [])
        return ids

    async def main():
        async with LocalCluster() as lc:
            lc.tenant("t")
            FakeNode.allocate = over_allocate
            try:
                code, body = await lc.add("default", "t", 1)
            finally:
                FakeNode.allocate = orig
            assert code == 500, body
            assert "ledger inconsistent" in body.get("error", ""), body
            assert await lc.audit("default", "t") == []
            node = lc.nodes["node-0"].node
            (c,) = [c for c in node.containers.values() if c.pod_name == "t"]
            assert node.container_devices(c.id) == []
            await asyncio.sleep(0.05)
            assert lc.cluster.placeholders() == [] and node.allocated == {}
            code, body = await lc.add("default", "t", 1)        # consistent again
            assert code == 200 and len(body["devices"]) == 1
    asyncio.run(main())


def test_fake_scheduler_admits_a_pod_once_despite_queued_retries():
    """Several capacity-freed retries queued for one unschedulable pod bind and admit it once
    (the fake kubelet Allocated it once per retry before: 3 devices for a 1-GPU pod)."""
    from gpumounter_amd.fakes.harness import LocalCluster

    async def main():
        async with LocalCluster() as lc:
            api = lc.cluster
            node = lc.nodes["node-0"].node
            body = {"metadata": {"name": "p", "namespace": "gpu-pool"},
                    "spec": {"containers": [{"name": "c", "image": "pause",
                                             "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
            api.create_pod("gpu-pool", body)
            await asyncio.sleep(0.05)
            for _ in range(3):                                   # queued retries
                api._spawn(api._schedule("gpu-pool", "p"))      # noqa: SLF001
            await asyncio.sleep(0.1)
            held = [d for d, (ns, pod, _) in node.allocated.items() if pod == "p"]
            assert len(held) == 1, node.allocated
    asyncio.run(main())
