"""C++ native layer through its Python bindings: sanitized unit tests, the amdsmi shim against the
mock (default + JSON-configured inventories, live process table), device-node injection (real
mknod as root, emulated markers, symlink-escape refusal), cgroup path resolution for every
driver/runtime/QoS/version combination, and the v1/v2 backends."""
import json
import os
import stat
import subprocess
import sys

import pytest

from gpumounter_amd import _native
from gpumounter_amd.fakes.node import FakeNode
from gpumounter_amd.models.device import DeviceNode
from gpumounter_amd.models.pod import ContainerRef
from gpumounter_amd.node import bpfvm
from gpumounter_amd.node.cgroup import (CgroupError, CgroupResolver, V1Backend,
                                        V2RecordingBackend, build_program)
from gpumounter_amd.node.devnodes import DevNodeError, DevNodeWriter, Target

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_unit_tests_under_asan_ubsan():
    res = subprocess.run(["make", "-C", os.path.join(ROOT, "native"), "check"],
                         capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert "native tests OK" in res.stdout


# ----------------------------------------------------------------------------------- amdsmi
def test_mock_inventory_default_mi355x_node(mock_inventory):
    inv = mock_inventory
    gpus = inv.gpus()
    assert len(gpus) == 8
    assert all(g.gfx_target == "gfx950" and g.market_name == "AMD Instinct MI355X" for g in gpus)
    assert [g.render_minor for g in gpus] == list(range(128, 136))
    assert [g.numa_node for g in gpus] == [0] * 4 + [1] * 4
    assert len({g.xgmi_hive_id for g in gpus}) == 1
    assert gpus[0].vram_bytes == 294896 * 2 ** 20   # 288 GB HBM3E
    links = inv.links()
    assert all(links.types[i][j] == (0 if i == j else 2) for i in range(8) for j in range(8))
    # the shim initialises amdsmi exactly once per process (reference re-inits per query)
    assert _native.mock_smi().gm_mock_init_calls() == 1


def test_mock_process_table_is_live(mock_inventory, tmp_path, monkeypatch):
    # processes come from the file named by procs_file / GM_AMDSMI_MOCK_PROCS, re-read per call;
    # the session mock was opened without one, so exercise the file path in a subprocess
    cfg = tmp_path / "mock.json"
    procs = tmp_path / "procs"
    cfg.write_text(json.dumps({
        "gpus": [{"bdf": "0000:11:00.0", "render": 140, "card": 1, "numa": 0, "hive": 7},
                 {"bdf": "0000:12:00.0", "render": 141, "card": 2, "numa": 1, "hive": 7},
                 {"bdf": "0000:21:00.0", "render": 142, "card": 3, "numa": 1, "hive": 9}],
        "links": {"overrides": [{"a": 0, "b": 1, "type": 2, "hops": 1, "weight": 20}]},
        "procs_file": str(procs)}))
    procs.write_text("1 4242 1024 python\n0 99 0 x\n")
    code = (
        "import sys, json; sys.path.insert(0, %r)\n"
        "from gpumounter_amd.hw.inventory import Inventory\n"
        "inv = Inventory('mock')\n"
        "print(json.dumps({'n': inv.count, 'r': [g.render_minor for g in inv.gpus()],"
        " 't': inv.links().types, 'p1': [p.pid for p in inv.processes(1)],"
        " 'p2': [p.pid for p in inv.processes(2)]}))\n" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env={**os.environ, "GM_AMDSMI_MOCK_CONFIG": str(cfg)}, timeout=60)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["n"] == 3 and d["r"] == [140, 141, 142]
    assert d["t"][0][1] == 2 and d["t"][0][2] == 1  # cross-hive pair falls back to PCIe
    assert d["p1"] == [4242] and d["p2"] == []


def test_mock_init_failure_reported(tmp_path):
    cfg = tmp_path / "bad.json"
    cfg.write_text(json.dumps({"fail_init": 34}))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from gpumounter_amd.hw.inventory import Inventory, InventoryError\n"
            "try:\n    Inventory('mock')\nexcept InventoryError as e:\n    print('ERR', e)\n"
            % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env={**os.environ, "GM_AMDSMI_MOCK_CONFIG": str(cfg)}, timeout=60)
    assert "ERR" in out.stdout and "DRIVER_NOT_LOADED" in out.stdout, out.stdout + out.stderr


# ----------------------------------------------------------------------------------- devnodes
NODES = [DeviceNode("/dev/kfd", 511, 0), DeviceNode("/dev/dri/renderD130", 226, 130),
         DeviceNode("/dev/dri/card2", 226, 2)]


@pytest.mark.parametrize("mode", ["emulate", "procroot"])
def test_devnodes_create_idempotent_remove(tmp_path, mode):
    if mode == "procroot" and os.geteuid() != 0:
        pytest.skip("mknod of a character device needs CAP_MKNOD (a GPU box runs as a user)")
    root = tmp_path / "root"
    (root / "dev").mkdir(parents=True)
    w = DevNodeWriter(mode)
    t = Target(root=str(root))
    assert w.create(t, NODES) == [0, 0, 0]
    assert w.create(t, NODES) == [1, 1, 1]
    for n in NODES:
        assert w.present(t, n)
        p = root / n.path.lstrip("/")
        st = os.lstat(p)
        assert stat.S_IMODE(st.st_mode) == 0o666
        if os.geteuid() == 0 and mode == "procroot":
            assert stat.S_ISCHR(st.st_mode) and os.major(st.st_rdev) == n.major
    assert w.remove(t, NODES) == [0, 0, 0]
    assert w.remove(t, NODES) == [1, 1, 1]
    assert not (root / "dev/kfd").exists()


def test_devnodes_refuse_symlink_escape(tmp_path):
    root = tmp_path / "root"
    outside = tmp_path / "outside"
    outside.mkdir()
    (root).mkdir()
    os.symlink(str(outside), root / "dev")  # hostile container: /dev → host dir
    w = DevNodeWriter("emulate")
    with pytest.raises(DevNodeError):
        w.create(Target(root=str(root)), [NODES[0]])
    assert os.listdir(outside) == []


def test_devnodes_never_clobber_foreign_file(tmp_path):
    root = tmp_path / "root"
    (root / "dev" / "dri").mkdir(parents=True)
    (root / "dev" / "dri" / "renderD130").write_text("tenant data")
    w = DevNodeWriter("emulate")
    with pytest.raises(DevNodeError):
        w.create(Target(root=str(root)), [NODES[1]])
    with pytest.raises(DevNodeError):
        w.remove(Target(root=str(root)), [NODES[1]])
    assert (root / "dev" / "dri" / "renderD130").read_text() == "tenant data"


def test_devnodes_procroot_by_pid_of_own_process():
    """Target by PID resolves /proc/<pid>/root (here: our own root) — read-only stat check."""
    w = DevNodeWriter("procroot")
    kind, ma, mi, _ = w.stat(Target(pid=os.getpid()), "/dev/null")
    assert (kind, ma, mi) == (1, 1, 3)
    with pytest.raises(DevNodeError):
        w.create(Target(pid=0), NODES[:1])  # empty container: clear error, no panic


# ----------------------------------------------------------------------------------- cgroups
def _pod(uid="1234-abcd", qos="besteffort"):
    res = {}
    if qos == "guaranteed":
        res = {"limits": {"cpu": "1", "memory": "1Gi"}, "requests": {"cpu": "1", "memory": "1Gi"}}
    elif qos == "burstable":
        res = {"requests": {"cpu": "100m"}}
    return {"metadata": {"uid": uid, "name": "p", "namespace": "ns"},
            "spec": {"containers": [{"name": "c", "resources": res}]}, "status": {}}


@pytest.mark.parametrize("mode", ["v1", "v2"])
@pytest.mark.parametrize("driver", ["cgroupfs", "systemd"])
@pytest.mark.parametrize("runtime", ["docker", "containerd", "cri-o"])
@pytest.mark.parametrize("qos", ["guaranteed", "burstable", "besteffort"])
def test_cgroup_resolution_matrix(tmp_path, mode, driver, runtime, qos, mock_inventory):
    node = FakeNode("n", str(tmp_path), mock_inventory.gpus(), cgroup_mode=mode,
                    cgroup_driver=driver, runtime=runtime)
    pod = _pod(qos=qos)
    ctr = node.start_container(pod, "c", [os.getpid()])
    r = CgroupResolver(node.cgroup_root)      # auto-detect mode and driver
    assert r.mode == mode
    d = r.container_dir(pod, ContainerRef("c", runtime, ctr.id, True))
    assert d == ctr.cgroup_dir
    assert r.pids(d) == [os.getpid()]
    if driver == "systemd":
        assert d.endswith(".scope")


def test_cgroup_resolution_via_proc_fallback(tmp_path):
    """Unknown kubelet layout: the container's cgroup is found through /proc/<pid>/cgroup."""
    root = tmp_path / "cg"
    odd = root / "custom.slice" / "my-runtime-abc123def.scope"
    odd.mkdir(parents=True)
    (root / "cgroup.controllers").write_text("cpu io memory\n")
    proc = tmp_path / "proc"
    (proc / "4242").mkdir(parents=True)
    (proc / "4242" / "cgroup").write_text("0::/custom.slice/my-runtime-abc123def.scope\n")
    (proc / "self").mkdir()
    r = CgroupResolver(str(root), proc_root=str(proc))
    assert r.mode == "v2"
    d = r.container_dir(_pod(), ContainerRef("c", "containerd", "abc123def", True))
    assert d == str(odd)


def test_cgroup_resolution_missing_raises(tmp_path, mock_inventory):
    FakeNode("n", str(tmp_path), mock_inventory.gpus())
    r = CgroupResolver(os.path.join(str(tmp_path), "cgroup"))
    with pytest.raises(CgroupError):
        r.container_dir(_pod(), ContainerRef("c", "containerd", "deadbeef", True))


def test_v1_backend_writes_kernel_rule_syntax(tmp_path, mock_inventory):
    node = FakeNode("n", str(tmp_path), mock_inventory.gpus(), cgroup_mode="v1")
    ctr = node.start_container(_pod(), "c")
    be = V1Backend()
    be.apply(ctr.cgroup_dir, NODES, [], NODES)
    assert open(os.path.join(ctr.cgroup_dir, "devices.allow")).read().splitlines() == [
        "c 511:0 rw", "c 226:130 rw", "c 226:2 rw"]
    assert be.allowed(ctr.cgroup_dir) == {(511, 0), (226, 130), (226, 2)}
    be.apply(ctr.cgroup_dir, [], NODES[1:], NODES[:1])
    assert open(os.path.join(ctr.cgroup_dir, "devices.deny")).read().splitlines() == [
        "c 226:130 rw", "c 226:2 rw"]
    assert be.allowed(ctr.cgroup_dir) == {(511, 0)}


def test_v2_recording_backend_program_semantics(tmp_path, mock_inventory):
    node = FakeNode("n", str(tmp_path), mock_inventory.gpus(), cgroup_mode="v2")
    ctr = node.start_container(_pod(), "c")
    be = V2RecordingBackend()
    be.apply(ctr.cgroup_dir, NODES, [], NODES)
    st = json.load(open(os.path.join(ctr.cgroup_dir, "gm.bpf.json")))
    assert st["mode"] == "set"
    prog = [int(x, 16) for x in st["insns"]]
    table = {tuple(e[:3]): e[3] for e in st["set"]}
    allowed = bpfvm.allowed_pairs(prog, [(511, 0), (226, 130), (226, 2), (226, 131), (1, 3),
                                         (1, 1)], maps={0: table})
    assert allowed == {(511, 0), (226, 130), (226, 2), (1, 3)}  # ours + runtime's /dev/null
    assert be.allowed(ctr.cgroup_dir) == {(511, 0), (226, 130), (226, 2)}
    be.apply(ctr.cgroup_dir, [], NODES, [])
    assert be.allowed(ctr.cgroup_dir) == set()
    assert build_program(NODES[:1], chained=False)[-1] == build_program(NODES, chained=False)[-1]


def test_host_pid_helpers():
    from gpumounter_amd.node import procs

    p = subprocess.Popen(["sleep", "30"])
    try:
        st = procs.start_time(p.pid)
        assert st > 0 and procs.same_process(p.pid, st)
        assert not procs.same_process(p.pid, st + 1)       # another process with that number
    finally:
        p.kill()
        p.wait()
    assert not procs.same_process(p.pid, st)               # exited and reaped
    assert procs.start_time(2 ** 22 + 7) == 0              # no such process
    assert not hasattr(procs, "signal_pids") and not hasattr(procs, "terminate")
    # /dev/null users: our own stdin/stdout may or may not be /dev/null; open one to be sure
    fd = os.open("/dev/null", os.O_RDONLY)
    try:
        assert os.getpid() in procs.filter_dev_users([os.getpid(), 1], 1, 3)
    finally:
        os.close(fd)


def test_scan_devs_reads_each_fd_table_once_for_many_devices():
    from gpumounter_amd.node import procs

    fz = os.open("/dev/zero", os.O_RDONLY)
    sleeper = subprocess.Popen(["sleep", "30"], stdin=subprocess.DEVNULL)
    try:
        hits, unreadable = procs.scan_devs([os.getpid(), sleeper.pid, 2 ** 22 + 9],
                                           [(1, 5), (1, 7), (1, 3)])
        assert hits[0][0] and not hits[0][1]              # we hold /dev/zero, not /dev/full
        assert hits[1][2] and not hits[1][0]              # the sleeper's stdin is /dev/null
        assert hits[2] == [False, False, False]           # exited PID: holds nothing
        assert unreadable == []
    finally:
        os.close(fz)
        sleeper.kill()
        sleeper.wait()


def test_busy_pids_auto_skips_amdsmi_when_fd_tables_are_readable(mock_inventory):
    from gpumounter_amd.node import procs

    inv = mock_inventory
    calls = []
    real = inv.processes

    def spy(i, *a, **k):
        calls.append(i)
        return real(i, *a, **k)
    inv.processes = spy
    try:
        g = inv.gpus()[0]
        assert procs.busy_pids(inv, [g], [os.getpid()], mode="auto") == {}
        assert calls == []                                 # fd scan was conclusive
        procs.busy_pids(inv, [g], [os.getpid()], mode="both")
        assert calls == [g.index]
    finally:
        inv.processes = real


def test_roctx_markers_are_safe_without_profiler():
    from gpumounter_amd.utils import trace

    with trace.span("outer", a=1) as s:
        with trace.span("inner"):
            trace.mark("tick")
    assert s.children[0].name == "inner" and s.duration_ms >= 0
    assert "inner" in s.flat()


def test_devnodes_bind_mode_policy(tmp_path):
    """Which containers get bind-mounted nodes (GM_DEV_BIND): auto = those whose process is in
    a user namespace other than the worker's (read from <proc_root>/<pid>/ns/user), with the
    nodes owned by the container's mapped root (uid_map/gid_map entry for id 0). The kernel
    side is tests/test_privileged_userns.py."""
    proc = tmp_path / "proc"
    for pid in ("self", "100", "200"):
        (proc / pid / "ns").mkdir(parents=True)
    os.link(__file__, proc / "self/ns/user")          # same inode as the worker: host userns
    os.link(__file__, proc / "100/ns/user")
    (proc / "200/ns/user").write_text("")            # another user namespace
    (proc / "200/uid_map").write_text("         0     165536      65536\n")
    (proc / "200/gid_map").write_text("         0     165536      65536\n")
    auto = DevNodeWriter("procroot", userns="auto", stage_dir=str(tmp_path / "st"),
                         proc_root=str(proc))
    assert not auto._bind(Target(pid=100))
    assert auto._bind(Target(pid=200))
    assert not auto._bind(Target(pid=300))            # gone: nothing to decide
    assert not auto._bind(Target(root=str(tmp_path)))  # hermetic root
    assert auto._mapped_root(Target(pid=200)) == (165536, 165536)
    assert auto._mapped_root(Target(pid=100)) == (-1, -1)
    off = DevNodeWriter("procroot", userns="off", proc_root=str(proc))
    assert not off._bind(Target(pid=200))
    assert DevNodeWriter("procroot", userns="bind", proc_root=str(proc))._bind(Target(pid=100))
    # emulate (unprivileged hermetic runs) never binds in auto mode
    assert not DevNodeWriter("emulate", userns="auto", proc_root=str(proc))._bind(
        Target(pid=200))
    # bind mode without a staging directory is refused before any native call
    with pytest.raises(DevNodeError, match="staging"):
        DevNodeWriter("procroot", userns="bind", proc_root=str(proc)).create(
            Target(pid=200), NODES[:1])


def test_tenant_view_library_resolves_through_emulated_state(tmp_path):
    """libgm_tenant_view.so: a GPU path is ENOENT without a node in the tenant rootfs, EPERM
    without a grant in the recorded allow set, and otherwise reaches the host node with that
    major:minor (ENXIO here: no GPU in this container); other paths are untouched."""
    import errno
    import json

    from gpumounter_amd.ops import tenant

    root, cg = tmp_path / "root", tmp_path / "cg"
    (root / "dev" / "dri").mkdir(parents=True)
    cg.mkdir()
    paths = ["/dev/kfd", "/dev/dri/renderD128", "/dev/null"]
    got = tenant.can_open(str(root), paths, str(cg))
    assert got == {"/dev/kfd": errno.ENOENT, "/dev/dri/renderD128": errno.ENOENT,
                   "/dev/null": 0}
    (root / "dev" / "kfd").write_text("gm-chr 511:0\n")
    (root / "dev" / "dri" / "renderD128").write_text("gm-chr 226:128\n")
    got = tenant.can_open(str(root), paths[:2], str(cg))
    assert set(got.values()) == {errno.EPERM}
    (cg / "gm.bpf.json").write_text(json.dumps({"set": [[2, 511, 0, 6], [2, 226, 128, 2]]}))
    got = tenant.can_open(str(root), paths[:2], str(cg))
    assert got["/dev/dri/renderD128"] == errno.EPERM          # read-only grant: not rw
    assert got["/dev/kfd"] in (0, errno.ENXIO)                 # granted: the host's node
    env = tenant.tenant_env(str(root), str(cg))
    assert env["LD_PRELOAD"].endswith("libgm_tenant_view.so")


def test_emulated_markers_appear_whole_and_leave_no_temporaries(tmp_path):
    """Without CAP_MKNOD (an unprivileged GPU box) emulate mode writes marker files. A marker is
    written under a hidden name and linked into place: created in place, a worker killed
    between the create and the write left an empty file that read as someone else's and was
    never replaced (chaos on the GPU box: nodes missing for good, "mknod failed: File
    exists")."""
    import shutil
    setpriv = shutil.which("setpriv")
    if setpriv is None or os.geteuid() != 0:
        pytest.skip("needs root and setpriv to drop CAP_MKNOD")
    root = tmp_path / "root"
    (root / "dev").mkdir(parents=True)
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from gpumounter_amd.node.devnodes import DevNodeWriter, Target\n"
        "from gpumounter_amd.models.device import DeviceNode\n"
        "nodes = [DeviceNode('/dev/kfd', 511, 0), DeviceNode('/dev/dri/renderD130', 226, 130)]\n"
        "w = DevNodeWriter('emulate'); t = Target(root=%r)\n"
        "print(w.create(t, nodes), w.create(t, nodes), [w.present(t, n) for n in nodes])\n"
        % (ROOT, str(root)))
    out = subprocess.run([setpriv, "--bounding-set=-mknod", "--inh-caps=-mknod", "--",
                          sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split("\n")[0] == "[0, 0] [1, 1] [True, True]", out.stdout
    for p, want in ((root / "dev/kfd", "gm-chr 511:0"),
                    (root / "dev/dri/renderD130", "gm-chr 226:130")):
        assert stat.S_ISREG(os.lstat(p).st_mode) and open(p).read().strip() == want
    left = [f for d in (root / "dev", root / "dev/dri") for f in os.listdir(d)
            if f.startswith(".")]
    assert left == []
