"""systemd DeviceAllow= persistence: the C++ D-Bus client (native/src/gm_sdbus.cpp) against an
independent fake systemd, the coalescing sync policy, and the full attach/detach path on a
systemd-driver node (systemd re-applies its own device policy on re-realise)."""
import asyncio
import ctypes as C
import os
import shutil
import tempfile

import pytest

from gpumounter_amd import _native
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.fakes.systemd_bus import FakeSystemd, unit_path
from gpumounter_amd.node.systemd import (DeviceAllowSync, SystemdBus, SystemdError, find_bus,
                                         maybe_wrap, unit_of)

UNIT = "cri-containerd-3f9a0c.scope"


@pytest.fixture(params=["private", "bus"])
def fake(request):
    d = tempfile.mkdtemp(prefix="gm-sd-")
    # systemd's private socket is recognised by its path; anything else is a message bus
    name = "systemd/private" if request.param == "private" else "system_bus_socket"
    os.makedirs(os.path.dirname(os.path.join(d, name)), exist_ok=True)
    fs = FakeSystemd(os.path.join(d, name), mode=request.param).start()
    fs.add_unit(UNIT, [("/dev/null", "rwm"), ("char-pts", "rwm")])
    yield fs
    fs.stop()
    shutil.rmtree(d, ignore_errors=True)


def test_unit_object_path_encoding_matches_sd_bus():
    buf = C.create_string_buffer(256)
    for unit in (UNIT, "docker-0.scope", "9lives.service", "crio-a_b.scope"):
        n = _native.host().gm_sd_unit_path(unit.encode(), buf, 256)
        assert n > 0 and buf.value.decode() == unit_path(unit)
    assert buf.value.decode().endswith("crio_2da_5fb_2escope")


def test_get_append_reset_roundtrip(fake):
    bus = SystemdBus(fake.path)
    assert bus.device_allow(UNIT) == [("/dev/null", "rwm"), ("char-pts", "rwm")]
    bus.set_device_allow(UNIT, [("/dev/kfd", "rw"), ("/dev/dri/renderD128", "rw")], reset=False)
    assert bus.device_allow(UNIT)[-2:] == [("/dev/kfd", "rw"), ("/dev/dri/renderD128", "rw")]
    bus.set_device_allow(UNIT, [("/dev/null", "rwm")], reset=True)
    assert bus.device_allow(UNIT) == [("/dev/null", "rwm")]
    bus.set_device_allow(UNIT, [], reset=True)
    assert bus.device_allow(UNIT) == []
    assert ("SetUnitProperties", UNIT) in fake.calls


def test_dbus_errors_are_reported(fake):
    bus = SystemdBus(fake.path)
    with pytest.raises(SystemdError, match="NoSuchUnit"):
        bus.device_allow("missing.scope")
    fake.fail_next = "org.freedesktop.DBus.Error.AccessDenied"
    with pytest.raises(SystemdError, match="AccessDenied"):
        bus.set_device_allow(UNIT, [("/dev/kfd", "rw")], reset=False)
    with pytest.raises(SystemdError, match="connect"):
        SystemdBus(fake.path + ".nope").device_allow(UNIT)


def test_sync_touches_only_managed_paths(fake):
    sync = DeviceAllowSync(SystemdBus(fake.path), retry_s=0.01)
    try:
        sync.update(UNIT, ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/card0"], [])
        assert sync.flush()
        assert fake.units[UNIT] == [("/dev/null", "rwm"), ("char-pts", "rwm"),
                                    ("/dev/dri/card0", "rw"), ("/dev/dri/renderD128", "rw"),
                                    ("/dev/kfd", "rw")]
        # coalescing: two updates before the thread runs collapse into the latest state
        sync.update(UNIT, ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/card0",
                           "/dev/dri/renderD129", "/dev/dri/card1"], [])
        sync.update(UNIT, ["/dev/kfd", "/dev/dri/renderD129", "/dev/dri/card1"],
                    ["/dev/dri/renderD128", "/dev/dri/card0"])
        assert sync.flush()
        assert fake.units[UNIT] == [("/dev/null", "rwm"), ("char-pts", "rwm"), ("/dev/kfd", "rw"),
                                    ("/dev/dri/card1", "rw"), ("/dev/dri/renderD129", "rw")]
        sync.update(UNIT, [], ["/dev/kfd", "/dev/dri/renderD129", "/dev/dri/card1"])
        assert sync.flush()
        assert fake.units[UNIT] == [("/dev/null", "rwm"), ("char-pts", "rwm")]   # runtime's own
        n = len(fake.calls)
        sync.update(UNIT, [], ["/dev/kfd"])                 # nothing to change: read only
        assert sync.flush() and [c[0] for c in fake.calls[n:]] == ["Get"]
        # a failed call is retried
        fake.fail_next = "org.freedesktop.DBus.Error.NoReply"
        sync.update(UNIT, ["/dev/kfd"], [])
        assert sync.flush()
        assert ("/dev/kfd", "rw") in fake.units[UNIT] and sync.errors == 1
    finally:
        sync.stop()


def test_unit_detection_and_policy(tmp_path, monkeypatch):
    from gpumounter_amd.node import systemd as sd
    from gpumounter_amd.node.cgroup import DeviceRuleBackend

    class Null(DeviceRuleBackend):
        name = "null"

        def apply(self, cgdir, grant, revoke, desired):
            pass

        def allowed(self, cgdir):
            return set()

    assert unit_of("/sys/fs/cgroup/kubepods.slice/kubepods-pod1.slice/cri-containerd-ab.scope") \
        == "cri-containerd-ab.scope"
    assert unit_of("/sys/fs/cgroup/devices/kubepods/pod1/abcdef") is None
    inner = Null()
    assert maybe_wrap(inner, "off", "", "systemd") is inner
    assert maybe_wrap(inner, "auto", "", "cgroupfs") is inner
    w = maybe_wrap(inner, "auto", str(tmp_path / "sock"), "systemd")
    assert isinstance(w, sd.SystemdPersistingBackend) and w.name == "null+systemd"
    w.sync.stop()
    monkeypatch.setattr(sd, "DEFAULT_BUSES", (str(tmp_path / "absent"),))
    assert find_bus("") is None
    assert maybe_wrap(inner, "auto", "", "auto") is inner
    with pytest.raises(SystemdError, match="no systemd bus"):
        maybe_wrap(inner, "on", "", "systemd")


def test_attach_detach_on_systemd_driver_node_keeps_scope_device_allow_in_step():
    d = tempfile.mkdtemp(prefix="gm-sd-")
    fs = FakeSystemd(os.path.join(d, "private"), auto_units=True).start()

    async def body(lc):
        worker = lc.nodes["node-0"].worker
        assert worker.backend.name.endswith("+systemd")
        lc.tenant("t")
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        assert worker.backend.sync.flush()
        (unit,) = [u for u in fs.units]
        assert unit.endswith(".scope")
        paths = [p for p, _ in fs.units[unit]]
        assert paths[:len(FakeSystemd.RUNTIME_DEFAULT)] == [p for p, _ in
                                                           FakeSystemd.RUNTIME_DEFAULT]
        ours = paths[len(FakeSystemd.RUNTIME_DEFAULT):]
        assert "/dev/kfd" in ours and len([p for p in ours if "renderD" in p]) == 2
        code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
        assert code == 200
        assert worker.backend.sync.flush()
        ours = [p for p, _ in fs.units[unit]][len(FakeSystemd.RUNTIME_DEFAULT):]
        assert len([p for p in ours if "renderD" in p]) == 1 and "/dev/kfd" in ours
        code, _ = await lc.remove("default", "t", [b["devices"][1]["uuid"]])
        assert code == 200
        assert worker.backend.sync.flush()
        assert fs.units[unit] == FakeSystemd.RUNTIME_DEFAULT
        assert await lc.audit("default", "t") == []

    async def main():
        async with LocalCluster(cgroup_mode="v2", cgroup_driver="systemd",
                                worker_overrides={"systemd_bus": fs.path}) as lc:
            await body(lc)
    try:
        asyncio.run(main())
    finally:
        fs.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_persisting_wrapper_forwards_every_backend_query():
    """The wrapper must answer every DeviceRuleBackend query from the backend it wraps: the
    base class's fallbacks (``installed`` = the effective verdict) would make the journal drop a
    grant a foreign program vetoes, on exactly the nodes where the wrapper is on."""
    import inspect

    from gpumounter_amd.node.cgroup import DeviceRuleBackend
    from gpumounter_amd.node.systemd import SystemdPersistingBackend

    class Inner(DeviceRuleBackend):
        name = "inner"

        def apply(self, cgdir, grant, revoke, desired):
            pass

        def allowed(self, cgdir):
            return set()                      # vetoed

        def installed(self, cgdir):
            return {(226, 128)}               # still ours

        def prune(self):
            return 7

    w = SystemdPersistingBackend(Inner(), sync=None)
    assert w.installed("/cg") == {(226, 128)} and w.allowed("/cg") == set() and w.prune() == 7
    queries = {n for n, f in inspect.getmembers(DeviceRuleBackend, inspect.isfunction)
               if not n.startswith("_")}
    assert queries <= set(vars(SystemdPersistingBackend)), \
        queries - set(vars(SystemdPersistingBackend))
