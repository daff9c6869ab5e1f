"""Pure-logic unit tests: config layering, pod helpers (QoS, quantities, container ids), the gRPC
schema's wire compatibility with the reference api.proto, and device-model helpers."""
import re

import pytest

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.api import podresources as pr
from gpumounter_amd.api.protodef import fields_of
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.device import AmdGpu, find_gpu, normalize_device_id
from gpumounter_amd.utils.config import Config

# ----------------------------------------------------------------------------------- config


def test_config_defaults_match_reference_ports_and_names():
    c = Config.load(env={})
    assert (c.master_port, c.worker_port) == (8080, 1200)        # main.go:237, worker main.go:24
    assert c.pool_namespace == "gpu-pool"                         # types.go:18
    assert c.worker_label == "app=gpu-mounter-worker"             # master main.go:256
    assert c.kubelet_socket == "/var/lib/kubelet/pod-resources/kubelet.sock"  # types.go:6-7
    assert c.resource_name == "amd.com/gpu"


def test_config_layering_yaml_env_overrides(tmp_path):
    f = tmp_path / "gm.yaml"
    f.write_text("worker_port: 1300\ncgroup_mode: v1\ntopology_policy: first-fit\nfoo: 1\n")
    env = {"GM_CONFIG": str(f), "GM_WORKER_PORT": "1400", "CGROUP_DRIVER": "systemd",
           "NODE_NAME": "n7", "GM_ROCTX": "false", "GM_KILL_GRACE_S": "2.5"}
    c = Config.load(env=env, master_port=9000)
    assert c.worker_port == 1400          # env beats file
    assert c.cgroup_mode == "v1"          # file
    assert c.cgroup_driver == "systemd"   # reference env name honoured
    assert c.node_name == "n7"
    assert c.roctx is False and c.kill_grace_s == 2.5
    assert c.master_port == 9000          # explicit override
    assert c.extra == {"foo": 1}


@pytest.mark.parametrize("bad", [{"GM_CGROUP_MODE": "v3"}, {"GM_DEVNODE_MODE": "x"},
                                 {"GM_WORKER_PORT": "-1"}, {"GM_WORKER_PORT": "70000"},
                                 {"GM_ROCTX": "maybe"}, {"GM_DEVNODE_USERNS": "maybe"}])
def test_config_rejects_invalid(bad):
    with pytest.raises(ValueError):
        Config.load(env=bad)


# ----------------------------------------------------------------------------------- pods


@pytest.mark.parametrize("q,v", [("100m", 0.1), ("1", 1), ("1Gi", 2 ** 30), ("2k", 2000),
                                 ("1.5", 1.5), ("1e3", 1000), ("512Mi", 512 * 2 ** 20)])
def test_parse_quantity(q, v):
    assert float(podu.parse_quantity(q)) == pytest.approx(v)


def _pod(*containers):
    return {"spec": {"containers": [{"name": f"c{i}", "resources": r}
                                    for i, r in enumerate(containers)]}, "status": {}}


@pytest.mark.parametrize("containers,qos", [
    ([{}], "BestEffort"),
    ([{"limits": {"cpu": "1", "memory": "1Gi"}}], "Guaranteed"),       # requests default to limits
    ([{"limits": {"cpu": "1", "memory": "1Gi"}, "requests": {"cpu": "1", "memory": "1Gi"}}],
     "Guaranteed"),
    ([{"limits": {"cpu": "2", "memory": "1Gi"}, "requests": {"cpu": "1", "memory": "1Gi"}}],
     "Burstable"),
    ([{"requests": {"cpu": "100m"}}], "Burstable"),
    ([{"limits": {"cpu": "1", "memory": "1Gi"}}, {}], "Burstable"),    # one container unset
    ([{"limits": {"amd.com/gpu": "1"}}], "BestEffort"),                # extended resources ignored
    ([{"limits": {"cpu": "1"}}], "Burstable"),
])
def test_qos_classifier(containers, qos):
    pod = _pod(*containers)
    # kubelet defaults requests to limits when only limits are set
    for c in pod["spec"]["containers"]:
        lim = c["resources"].get("limits", {})
        c["resources"].setdefault("requests", {k: v for k, v in lim.items()
                                               if k in ("cpu", "memory")})
    assert podu.qos_class(pod) == qos


def test_container_id_runtimes_and_all_containers():
    pod = {"status": {"containerStatuses": [
        {"name": "a", "containerID": "docker://abc", "state": {"running": {}}},
        {"name": "b", "containerID": "containerd://def", "state": {"running": {}}},
        {"name": "c", "containerID": "cri-o://123", "state": {"waiting": {}}},
        {"name": "d"}]}}
    refs = podu.running_containers(pod)
    assert [(r.name, r.runtime, r.id, r.running) for r in refs] == [
        ("a", "docker", "abc", True), ("b", "containerd", "def", True),
        ("c", "cri-o", "123", False)]
    assert [r.name for r in podu.running_containers(pod, "b")] == ["b"]


def test_unschedulable_detection_any_condition():
    pod = {"status": {"conditions": [{"type": "Ready", "status": "False"},
                                     {"type": "PodScheduled", "status": "False",
                                      "reason": "Unschedulable", "message": "0/1 nodes"}]}}
    assert podu.is_unschedulable(pod) == "0/1 nodes"
    assert podu.is_unschedulable({"status": {}}) is None


# ----------------------------------------------------------------------------------- schema


def test_wire_bytes_identical_to_reference_encoding():
    # golden bytes produced for the reference's AddGPURequest{pod_name:"p", namespace:"default",
    # gpu_num:2} (SURVEY §0.1 probe)
    r = api.AddGPURequest(pod_name="p", namespace="default", gpu_num=2)
    assert r.SerializeToString() == b"\n\x01p\x12\x07default\x18\x02"
    assert api.AddGPURequest.FromString(b"\n\x01p\x12\x07default\x18\x02 \x01").is_entire_mount


def test_reference_field_numbers_and_enums_preserved():
    assert fields_of(api.AddGPURequest)[:4] == [("pod_name", 1), ("namespace", 2),
                                                ("gpu_num", 3), ("is_entire_mount", 4)]
    assert fields_of(api.RemoveGPURequest)[:4] == [("pod_name", 1), ("namespace", 2),
                                                   ("uuids", 3), ("force", 4)]
    assert fields_of(api.AddGPUResponse)[0] == ("add_gpu_result", 1)
    assert fields_of(api.RemoveGPUResponse)[0] == ("remove_gpu_result", 1)
    assert (api.AddGPUResponse.Success, api.AddGPUResponse.InsufficientGPU,
            api.AddGPUResponse.PodNotFound) == (0, 1, 2)
    assert (api.RemoveGPUResponse.Success, api.RemoveGPUResponse.GPUBusy,
            api.RemoveGPUResponse.PodNotFound, api.RemoveGPUResponse.GPUNotFound) == (0, 1, 2, 4)
    assert api.ADD_GPU == "/gpu_mount.AddGPUService/AddGPU"
    assert api.REMOVE_GPU == "/gpu_mount.RemoveGPUService/RemoveGPU"


def test_proto_text_matches_runtime_descriptors():
    import os

    path = os.path.join(os.path.dirname(api.__file__), "gpu_mount.proto")
    text = open(path).read()
    for cls in (api.AddGPURequest, api.AddGPUResponse, api.RemoveGPURequest,
                api.RemoveGPUResponse, api.Device, api.StageTiming):
        body = re.search(r"message %s \{(.*?)\n\}" % cls.DESCRIPTOR.name, text, re.S).group(1)
        declared = {(m.group(2), int(m.group(3)))
                    for m in re.finditer(r"^\s+(repeated \S+|\S+) (\w+) = (\d+);", body, re.M)}
        assert declared == set(fields_of(cls)), cls.DESCRIPTOR.name


def test_podresources_v1_is_wire_compatible_with_v1alpha1():
    r = pr.V1.ListPodResourcesResponse()
    c = r.pod_resources.add(name="p", namespace="ns").containers.add(name="c")
    d = c.devices.add(resource_name="amd.com/gpu", device_ids=["0000:05:00.0"])
    d.topology.nodes.add(ID=1)
    old = pr.V1ALPHA1.ListPodResourcesResponse.FromString(r.SerializeToString())
    assert old.pod_resources[0].containers[0].devices[0].device_ids == ["0000:05:00.0"]


# ----------------------------------------------------------------------------------- device


def test_device_nodes_and_ledger_keys():
    g = AmdGpu(index=3, uuid="u-3", bdf="0000:75:00.0", render_minor=131, card_minor=3)
    nodes = g.device_nodes()
    assert [(n.path, n.major, n.minor) for n in nodes] == [
        ("/dev/dri/renderD131", 226, 131), ("/dev/dri/card3", 226, 3)]
    assert nodes[0].cgroup_rule() == "c 226:131 rw"
    for key in ("u-3", "0000:75:00.0", "75:00.0", "renderD131", "CARD3", "GPU-u-3"):
        assert find_gpu([g], key) is g, key
    assert normalize_device_id(" ABC ") == "abc"


def test_fast_to_dict_matches_json_format():
    """api/protodef.to_dict is the master's reply encoder; it must equal protobuf's MessageToDict
    (proto field names, all fields, enums by name, 64-bit ints as strings)."""
    from google.protobuf import json_format

    from gpumounter_amd.api import gpu_mount as api
    from gpumounter_amd.api.protodef import to_dict

    def ref(m):
        return json_format.MessageToDict(m, preserving_proto_field_name=True,
                                         always_print_fields_with_no_presence=True)
    msgs = [
        api.AddGPUResponse(),
        api.AddGPUResponse(add_gpu_result=api.ADD_INSUFFICIENT, message="x", total_ms=1.5,
                           devices=[api.Device(uuid="u", bdf="0000:05:00.0", index=3,
                                               render_minor=131, numa_node=1)],
                           timings=[api.StageTiming(name="mount", ms=0.25)]),
        api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_BUSY, killed_pids=[7, 9],
                              message="busy"),
        api.AddGPURequest(pod_name="p", namespace="n", gpu_num=2, is_entire_mount=True,
                          idempotency_key="k"),
        api.RemoveGPURequest(pod_name="p", namespace="n", uuids=["a", "b"], force=True),
    ]
    for m in msgs:
        assert to_dict(m) == ref(m), type(m).__name__


def test_probe_gemm_wrappers_validate_before_touching_the_gpu():
    """The GEMM wrappers reject what the kernels' grids assume away (tile multiples, dtype,
    layout) on the host, before any HIP call, so a bad shape can never reach a launch."""
    import pytest
    import torch

    from gpumounter_amd.ops import probe

    bf = torch.bfloat16
    cases = [
        (torch.zeros(256, 64, dtype=torch.float32), torch.zeros(256, 64, dtype=bf)),   # dtype
        (torch.zeros(256, 64, dtype=bf), torch.zeros(64, 256, dtype=bf).t()),          # layout
        (torch.zeros(250, 64, dtype=bf), torch.zeros(256, 64, dtype=bf)),              # M % 256
        (torch.zeros(256, 64, dtype=bf), torch.zeros(200, 64, dtype=bf)),              # N % 256
        (torch.zeros(256, 48, dtype=bf), torch.zeros(256, 48, dtype=bf)),              # K % 64
        (torch.zeros(256, 64, dtype=bf), torch.zeros(256, 128, dtype=bf)),             # K mismatch
    ]
    for a, bt in cases:
        with pytest.raises(probe.ProbeError):
            probe.gemm_nt(a, bt)
    a, bt = torch.zeros(256, 64, dtype=bf), torch.zeros(256, 64, dtype=bf)
    with pytest.raises(probe.ProbeError):
        probe.gemm_nt(a, bt, out=torch.zeros(256, 256, dtype=torch.float32))
    with pytest.raises(probe.ProbeError):
        probe.gemm_bf16(torch.zeros(64, 30, dtype=bf), torch.zeros(30, 64, dtype=bf))
    # the native entry points check their arguments before selecting a device
    for n, secs in ((300, 1.0), (256, 0.0), (-256, 1.0)):
        with pytest.raises(probe.ProbeError):
            probe.burn_in(0, secs, n)
    with pytest.raises(probe.ProbeError):
        probe.gemm_tflops(0, 256, 256, 100, 1)


def test_gc_pause_monitor_records_collections():
    import gc

    from gpumounter_amd.utils import runtime
    runtime.watch_gc_pauses(0.0)          # every collection counts at threshold 0
    runtime.watch_gc_pauses(0.0)          # idempotent: one callback
    n = len(runtime.gc_pauses)
    gc.collect()
    assert len(runtime.gc_pauses) == min(n + 1, 100)
    assert runtime.gc_pauses[-1][0] == 2


def test_tail_report_attributes_slow_cycles(tmp_path):
    import importlib.util
    import json
    import os

    spec = importlib.util.spec_from_file_location(
        "tail_report", os.path.join(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__))), "bench", "tail_report.py"))
    tr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tr)
    f = tmp_path / "s.jsonl"
    rows = [{"t": i * 0.01, "attach_ms": 1.0, "detach_ms": 1.0,
             "stages": {"ledger_reserve": 0.3, "mount": 0.2, "mount.devnodes": 0.1}}
            for i in range(99)]
    rows.append({"t": 1.0, "attach_ms": 80.0, "detach_ms": 1.0,
                 "stages": {"ledger_reserve": 79.0, "mount": 0.2, "mount.devnodes": 0.1}})
    f.write_text("".join(json.dumps(r) + "\n" for r in rows))
    rep = tr.report(str(f))
    assert rep["cycles"] == 100 and rep["attach_ms"]["max"] == 80.0
    top = rep["slowest"][0]
    assert top["largest"] == ["worker:ledger_reserve", 79.0]
    # sub-stages not summed: 1.0 - (0.3 + 0.2) outside the worker, as in every cycle
    assert rep["component_p50_ms"]["outside_worker"] == 0.5
    assert rep["tail_excess_over_p50_ms"]["worker:ledger_reserve"] == 78.7
    # with the master's stages recorded, the outside is split into HTTP / master / gRPC
    rows = [{"t": 0.0, "attach_ms": 2.0,
             "stages": {"ledger_reserve": 0.3, "mount": 0.2, "rpc_queue": 0.01, "rpc_tail": 0.04},
             "master": {"master_authz": 0.01, "master_locate": 0.01, "master_rpc": 1.7,
                        "master_payload": 0.03}}]
    f.write_text(json.dumps(rows[0]) + "\n")
    c = tr.report(str(f))["component_p50_ms"]
    assert c["client_http"] == 0.25 and c["master_own"] == 0.05 and c["worker_rpc"] == 0.05
    assert c["grpc"] == 1.15 and c["worker:ledger_reserve"] == 0.3


def test_informer_drops_write_through_older_than_a_relist():
    """after a relist the cache may hold a newer version than a write response whose
    request went out before it; that response must not overwrite it (the watch resumes from
    the list and never redelivers the newer version)."""
    from gpumounter_amd.cluster.informer import PodInformer

    inf = PodInformer(kube=None)

    def pod(rv, v, name="p", uid="u"):
        return {"metadata": {"namespace": "ns", "name": name, "uid": uid, "resourceVersion": rv,
                             "annotations": {"v": v}}}
    ep = inf.epoch
    inf.cache[("ns", "p")] = pod("12", "from-list")      # what the relist delivered
    inf.epoch += 1
    inf.upsert(pod("9", "our-older-patch"), ep)
    assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "from-list"
    inf.upsert(pod("13", "patch-after-relist"), inf.epoch)
    assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "patch-after-relist"
    inf.upsert(pod("14", "created", name="q", uid="w"), ep)   # not in the list: newer, kept
    assert inf.get("ns", "q") is not None


def test_informer_keeps_write_through_against_older_watch_events():
    """Our PATCH response is cached at once; watch events for that object older than it (the
    watch lags) must not overwrite it until the watch has delivered our version."""
    import asyncio

    from gpumounter_amd.cluster.informer import PodInformer

    def pod(rv, v):
        return {"metadata": {"namespace": "ns", "name": "p", "uid": "u", "resourceVersion": rv,
                             "annotations": {"v": v}}}

    class Feed(PodInformer):
        def __init__(self):
            super().__init__(kube=None)
            self.q = asyncio.Queue()

        async def _list(self):
            return [pod("1", "listed")], "1"

        async def _watch(self, timeout_s):
            while True:
                ev = await self.q.get()
                if ev is None:
                    return
                yield ev

    async def main():
        inf = Feed()
        await inf.start()
        inf.upsert(pod("5", "patched"), inf.epoch)         # our write, watch still at rv 1
        await inf.q.put(("MODIFIED", pod("3", "kubelet-status")))
        await asyncio.sleep(0.01)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "patched"
        await inf.q.put(("MODIFIED", pod("5", "patched")))  # the watch reaches our write
        await inf.q.put(("MODIFIED", pod("6", "later")))
        await asyncio.sleep(0.01)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "later"
        await inf.stop()
    asyncio.run(main())


def test_reserve_gate_shared_and_exclusive():
    """Ordinary reservations overlap; a placement correction (exclusive) waits for them, runs
    alone, and new ordinary ones queue behind a waiting correction (no starvation)."""
    import asyncio

    from gpumounter_amd.cluster.correction import ReserveGate as _SharedExclusive

    async def main():
        g = _SharedExclusive()
        log = []

        async def shared(tag, hold):
            async with g.shared():
                log.append(("in", tag))
                await asyncio.sleep(hold)
                log.append(("out", tag))

        async def exclusive(tag, hold):
            async with g.exclusive():
                log.append(("in", tag))
                await asyncio.sleep(hold)
                log.append(("out", tag))
        a = asyncio.ensure_future(shared("s1", 0.05))
        b = asyncio.ensure_future(shared("s2", 0.05))
        await asyncio.sleep(0.01)
        x = asyncio.ensure_future(exclusive("x", 0.03))
        await asyncio.sleep(0.01)
        c = asyncio.ensure_future(shared("s3", 0.01))
        await asyncio.gather(a, b, x, c)
        order = [e for e in log]
        assert order[:2] == [("in", "s1"), ("in", "s2")]            # overlapping
        ix = order.index(("in", "x"))
        assert ("out", "s1") in order[:ix] and ("out", "s2") in order[:ix]
        assert order[ix + 1] == ("out", "x")                        # alone
        assert order.index(("in", "s3")) > ix                      # queued behind x
    asyncio.run(main())


def test_informer_relist_resolves_our_unechoed_writes_with_a_get():
    """A relist served before our acknowledged PATCH holds an older version than the write, and
    a write-through that arrives after a relist cannot tell older from newer: in both cases the
    informer asks the apiserver (a GET is newer than both) instead of serving a stale object —
    a stale 'still a candidate' or 'still standby' view is what lets a reconciler release, or a
    pool claim twice, a GPU that is in use."""
    import asyncio

    from gpumounter_amd.cluster.informer import PodInformer

    def pod(rv, v):
        return {"metadata": {"namespace": "ns", "name": "p", "uid": "u", "resourceVersion": rv,
                             "annotations": {"v": v}}}

    server = {"obj": pod("1", "v1")}

    class Kube:
        gets = 0

        async def get_pod(self, ns, name):
            Kube.gets += 1
            return server["obj"]

    class Feed(PodInformer):
        def __init__(self):
            super().__init__(kube=Kube())
            self.q = asyncio.Queue()
            self.listed = [pod("1", "v1")]

        async def _list(self):
            return list(self.listed), "1"

        async def _watch(self, timeout_s):
            while True:
                ev = await self.q.get()
                if ev is None:
                    return
                yield ev

    async def main():
        inf = Feed()
        await inf.start()
        # our PATCH is acknowledged (rv 5); then a relist arrives that was served before it
        server["obj"] = pod("5", "patched")
        inf.upsert(pod("5", "patched"), inf.epoch)
        await inf._relist()                        # lists rv 1 (older than our write)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "patched"
        assert Kube.gets == 1
        # a write-through whose request went out before a relist: resolved by a GET as well
        ep = inf.epoch
        inf.listed = [pod("5", "patched")]
        await inf._relist()
        server["obj"] = pod("7", "patched-again")
        inf.upsert(pod("7", "patched-again"), ep)
        await asyncio.sleep(0.01)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "patched-again"
        # the resumed watch replays older events: skipped until it reaches the fetched version
        await inf.q.put(("MODIFIED", pod("6", "replayed-older")))
        await asyncio.sleep(0.01)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "patched-again"
        await inf.stop()
    asyncio.run(main())


def test_informer_relist_keeps_writes_acknowledged_while_it_was_in_flight():
    """A relist installs its list only after the GETs of its suspects, which a rate-limiting
    apiserver can stretch to hundreds of ms. A create and a PATCH of ours acknowledged in that
    window went into the cache the relist then replaced with a list served before them: the
    just-created placeholders vanished from the view, and a reconcile revoked the GPUs they had
    just had mounted (chaos seed 114). They stand in until a GET settles them."""
    import asyncio

    from gpumounter_amd.cluster.informer import PodInformer

    def pod(name, rv, v):
        return {"metadata": {"namespace": "ns", "name": name, "uid": "u-" + name,
                             "resourceVersion": rv, "annotations": {"v": v}}}

    server = {"a": pod("a", "1", "v1")}
    gate = asyncio.Event()

    class Kube:
        async def get_pod(self, ns, name):
            if name == "a" and not gate.is_set():
                await gate.wait()                   # the suspect's GET is slow
            if name not in server:
                from gpumounter_amd.cluster.kube import NotFound
                raise NotFound(404, name)
            return server[name]

    class Feed(PodInformer):
        def __init__(self):
            super().__init__(kube=Kube())
            self.listed = [pod("a", "1", "v1")]

        async def _list(self):
            return list(self.listed), "2"

        async def _watch(self, timeout_s):
            await asyncio.Event().wait()
            yield                                   # never delivers

    async def main():
        inf = Feed()
        await inf.start()
        inf.upsert(pod("a", "2", "ours"), inf.epoch)    # unechoed: a suspect of the relist
        inf.listed = [pod("a", "1", "v1")]
        relist = asyncio.ensure_future(inf._relist())
        await asyncio.sleep(0.01)                       # listed; its GET is in flight
        server["a"] = pod("a", "3", "patched")
        inf.upsert(pod("a", "3", "patched"), inf.epoch)     # acknowledged meanwhile
        server["b"] = pod("b", "4", "created")
        inf.upsert(pod("b", "4", "created"), inf.epoch)
        gate.set()
        await relist
        assert inf.get("ns", "b") is not None, "a create acknowledged during the relist is lost"
        await inf.wait_for(lambda: inf.settled, 1.0)
        assert inf.get("ns", "a")["metadata"]["annotations"]["v"] == "patched"
        assert inf.get("ns", "b")["metadata"]["annotations"]["v"] == "created"
        await inf.stop()
    asyncio.run(main())


def test_a_delete_of_ours_older_than_the_relist_is_not_read_as_foreign():
    """Our DELETE lands after a relist's list was served: the relist leaves the object out (its
    suspect GET found it gone), and the watch, resumed from the list's version, then delivers
    the DELETED event. Pruning the tombstone at the relist made that event a foreign delete: a
    revocation reaction under the owner (chaos seed 114, 'deleted externally' for a pick's
    surplus the attach had just released)."""
    import asyncio

    from gpumounter_amd.cluster.informer import PodInformer
    from gpumounter_amd.cluster.placeholder import PlaceholderManager

    async def main():
        inf = PodInformer(kube=None)
        ph = PlaceholderManager(None, None, None, inf, "node-0")
        foreign = []
        ph.on_foreign_delete.append(foreign.append)
        now = asyncio.get_running_loop().time()
        ph.tombstones["u1"] = now                                   # our DELETE just went out
        ph.tombstones["u0"] = now - ph.TOMBSTONE_KEEP_S - 1         # an old one, event missed
        ph._on_event("RELIST", {})                                   # the list holds neither
        assert "u0" not in ph.tombstones and "u1" in ph.tombstones
        ph._on_event("DELETED", {"metadata": {"namespace": "p", "name": "x", "uid": "u1"}})
        assert not foreign
    asyncio.run(main())


def test_informer_resolve_does_not_replace_a_newer_write_of_ours():
    """A GET that settles a key after a relist was sent before our next PATCH of that key and
    answers after it: its (older) object must not replace the PATCH's, or the cache would also
    skip the watch's event for the PATCH as older than what it holds."""
    import asyncio

    from gpumounter_amd.cluster.informer import PodInformer

    def pod(rv, v):
        return {"metadata": {"namespace": "ns", "name": "p", "uid": "u", "resourceVersion": rv,
                             "annotations": {"v": v}}}

    server = {"obj": pod("5", "first")}
    answers = []

    class Kube:
        async def get_pod(self, ns, name):
            obj = server["obj"]                     # read when the request is served...
            if not answers:
                answers.append(obj)
                await asyncio.sleep(0.05)           # ...answered late the first time
            return obj

    class Feed(PodInformer):
        def __init__(self):
            super().__init__(kube=Kube())

        async def _list(self):
            return [pod("1", "listed")], "1"

        async def _watch(self, timeout_s):
            await asyncio.Event().wait()
            yield

    async def main():
        inf = Feed()
        await inf.start()
        ep = inf.epoch
        await inf._relist()
        inf.upsert(pod("5", "first"), ep)           # overtaken by the relist: a GET settles it
        await asyncio.sleep(0.01)                   # the GET is served (rv 5), reply on its way
        server["obj"] = pod("6", "second")
        inf.upsert(pod("6", "second"), inf.epoch)   # our next PATCH, acknowledged first
        await inf.wait_for(lambda: inf.settled, 1.0)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "second"
        await inf.stop()
    asyncio.run(main())


def test_informer_relist_newer_than_our_write_does_not_stall_the_key():
    """The list holds a version newer than our unechoed write (someone wrote after us): the GET
    returns that same version, which the resumed watch will never deliver again — the key must
    not wait for it, or every later event for the object would be skipped for good."""
    import asyncio

    from gpumounter_amd.cluster.informer import PodInformer

    def pod(rv, v):
        return {"metadata": {"namespace": "ns", "name": "p", "uid": "u", "resourceVersion": rv,
                             "annotations": {"v": v}}}

    class Kube:
        async def get_pod(self, ns, name):
            return pod("8", "someone-else")

    class Feed(PodInformer):
        def __init__(self):
            super().__init__(kube=Kube())
            self.q = asyncio.Queue()
            self.listed = [pod("1", "v1")]

        async def _list(self):
            return list(self.listed), "8"

        async def _watch(self, timeout_s):
            while True:
                ev = await self.q.get()
                if ev is None:
                    return
                yield ev

    async def main():
        inf = Feed()
        await inf.start()
        inf.upsert(pod("5", "ours"), inf.epoch)
        inf.listed = [pod("8", "someone-else")]
        await inf._relist()
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "someone-else"
        await inf.q.put(("MODIFIED", pod("9", "next")))     # the next change arrives
        await asyncio.sleep(0.01)
        assert inf.get("ns", "p")["metadata"]["annotations"]["v"] == "next"
        await inf.stop()
    asyncio.run(main())
