"""Real-kernel enforcement tests for the device-access backends (root with mount + bpf; GM_PRIVILEGED_TESTS=0/1 forces off/on,
needs root with CAP_SYS_ADMIN/CAP_BPF). They mount a private cgroup2 hierarchy (or use the v1
devices controller), put a child process into a fresh cgroup, and check that the process can open
exactly the devices the backend granted — using harmless /dev/null, /dev/zero, /dev/full.

cgroup v2: a "runtime" program (allow /dev/null only) is attached first, exactly like runc does;
gm_bpf_dev_install then swaps in the gpumounter program that grants /dev/zero and tail-calls the
runtime program; gm_bpf_dev_restore puts the runtime program back.
"""
import ctypes as C
import os
import subprocess
import sys
import tempfile
import uuid

import pytest
from conftest import privileged_skip

from gpumounter_amd import _native
from gpumounter_amd.models.device import DeviceNode
from gpumounter_amd.node.cgroup import V1Backend, V2BpfBackend, _rule_array

pytestmark = [pytest.mark.privileged, privileged_skip()]

NULL, ZERO, FULL = DeviceNode("/dev/null", 1, 3), DeviceNode("/dev/zero", 1, 5), \
    DeviceNode("/dev/full", 1, 7)

PROBE = ("import sys\n"
         "out=[]\n"
         "for p in sys.argv[1:]:\n"
         "    try:\n"
         "        open(p,'rb').close(); out.append('1')\n"
         "    except OSError:\n"
         "        out.append('0')\n"
         "print(''.join(out))\n")


def can_open(cg_procs: str, paths):
    """Spawn a child, move it into the cgroup before it opens anything, report per-path access."""
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # child: wait until the parent moved us, then exec the probe
        os.close(w)
        os.read(r, 1)
        os.execv(sys.executable, [sys.executable, "-c", PROBE] + list(paths))
    os.close(r)
    with open(cg_procs, "w") as fh:
        fh.write(str(pid))
    out_r, out_w = os.pipe()
    os.close(out_r)
    os.close(out_w)
    os.write(w, b"x")
    os.close(w)
    _, status = os.waitpid(pid, 0)
    return status


def probe_access(cgdir, paths):
    code = (f"import os,sys\n"
            f"open({os.path.join(cgdir, 'cgroup.procs')!r},'w').write(str(os.getpid()))\n"
            + PROBE)
    res = subprocess.run([sys.executable, "-c", code] + list(paths), capture_output=True,
                         text=True, timeout=30)
    assert res.returncode == 0, res.stderr
    return res.stdout.strip()


@pytest.fixture
def bpffs():
    d = tempfile.mkdtemp(prefix="gm-bpffs-")
    subprocess.run(["mount", "-t", "bpf", "bpf", d], check=True)
    try:
        yield d
    finally:
        subprocess.run(["umount", d], check=True)
        os.rmdir(d)


@pytest.fixture
def cgroup2_child():
    mnt = tempfile.mkdtemp(prefix="gm-cg2-")
    subprocess.run(["mount", "-t", "cgroup2", "none", mnt], check=True)
    cg = os.path.join(mnt, "gm-test-" + uuid.uuid4().hex[:8])
    os.mkdir(cg)
    try:
        yield cg
    finally:
        # move anything left back to the root, then clean up
        try:
            with open(os.path.join(cg, "cgroup.procs")) as fh:
                for pid in fh.read().split():
                    with open(os.path.join(mnt, "cgroup.procs"), "w") as out:
                        out.write(pid)
        except OSError:
            pass
        os.rmdir(cg)
        subprocess.run(["umount", mnt], check=True)
        os.rmdir(mnt)


def attach_runtime_program(cg, name=b"runc_devices", nodes=((1, 3),)):
    """Mimic runc (or systemd): allow the given nodes rw + mknod, deny everything else,
    ALLOW_MULTI. Default: /dev/null only."""
    rules = _rule_array([_native.DevRule(b"c", 7, 1, 0, ma, mi) for ma, mi in nodes])
    lib = _native.host()
    need = -lib.gm_bpf_dev_build(rules, len(nodes), 0, -1, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build(rules, len(nodes), 0, -1, buf, need)
    fd = lib.gm_bpf_dev_load(buf, n, name, None, 0)
    assert fd >= 0, os.strerror(-fd)
    # BPF_PROG_ATTACH through a throwaway install path is not possible (ours would replace it),
    # so attach with raw syscall via ctypes
    import ctypes.util

    libc = C.CDLL(ctypes.util.find_library("c"), use_errno=True)
    cgfd = os.open(cg, os.O_RDONLY | os.O_DIRECTORY)
    attr = (C.c_uint8 * 128)()
    # union bpf_attr for BPF_PROG_ATTACH: target_fd, attach_bpf_fd, attach_type, attach_flags
    C.memmove(attr, (C.c_uint32 * 4)(cgfd, fd, 6, 2), 16)   # BPF_CGROUP_DEVICE=6, ALLOW_MULTI=2
    rc = libc.syscall(321, 8, attr, 128)  # __NR_bpf=321, BPF_PROG_ATTACH=8
    os.close(cgfd)
    assert rc == 0, os.strerror(C.get_errno())
    return fd


@pytest.mark.parametrize("pinned", [True, False])
def test_cgroup_v2_bpf_install_and_restore(cgroup2_child, bpffs, pinned):
    cg = cgroup2_child
    paths = [NULL.path, ZERO.path, FULL.path]
    assert probe_access(cg, paths) == "111"          # no program: unrestricted
    attach_runtime_program(cg)
    assert probe_access(cg, paths) == "100"          # runtime policy: only /dev/null
    be = V2BpfBackend(bpffs if pinned else "")
    be.apply(cg, [ZERO], [], [ZERO])                 # gpumounter grants /dev/zero
    assert probe_access(cg, paths) == "110"
    ids = (C.c_uint32 * 8)()
    n, flags = C.c_uint32(0), C.c_uint32(0)
    assert _native.host().gm_bpf_dev_query(cg.encode(), ids, 8, C.byref(n), C.byref(flags)) == 0
    assert n.value == 1                              # replaced, not stacked
    name = C.create_string_buffer(32)
    _native.host().gm_bpf_prog_name(ids[0], name, 32)
    assert name.value == b"gm_devallow"
    be.apply(cg, [FULL], [], [ZERO, FULL])           # update: chain target preserved
    assert probe_access(cg, paths) == "111"
    # audit reads the grants back from the kernel's xlated program
    assert be.allowed(cg) >= {(ZERO.major, ZERO.minor), (FULL.major, FULL.minor)}
    be.apply(cg, [], [ZERO], [FULL])                 # revoke /dev/zero
    assert probe_access(cg, paths) == "101"
    assert (ZERO.major, ZERO.minor) not in be.allowed(cg)
    be.apply(cg, [], [FULL], [])                     # last GPU gone: runtime program restored
    assert be.allowed(cg) == set()
    assert probe_access(cg, paths) == "100"
    _native.host().gm_bpf_dev_query(cg.encode(), ids, 8, C.byref(n), C.byref(flags))
    _native.host().gm_bpf_prog_name(ids[0], name, 32)
    assert n.value == 1 and name.value == b"runc_devices"
    assert not [f for f in os.listdir(bpffs) if f.startswith("gm_")]  # pin removed


def _names(cg):
    ids = (C.c_uint32 * 8)()
    n, flags = C.c_uint32(0), C.c_uint32(0)
    assert _native.host().gm_bpf_dev_query(cg.encode(), ids, 8, C.byref(n), C.byref(flags)) == 0
    out = []
    for i in range(n.value):
        name = C.create_string_buffer(32)
        _native.host().gm_bpf_prog_name(ids[i], name, 32)
        out.append(name.value.decode())
    return sorted(out)


def test_cgroup_v2_wraps_every_program_of_an_allow_multi_stack(cgroup2_child, bpffs):
    """systemd-driver hosts: runc's program and systemd's (from the scope's DeviceAllow) are both
    attached, and each can veto an access. Every one gets wrapped; a program systemd attaches
    later makes the audit report nothing granted until the reconciler wraps that one too."""
    cg = cgroup2_child
    paths = [NULL.path, ZERO.path, FULL.path]
    attach_runtime_program(cg, b"runc_devices", ((1, 3), (1, 7)))     # null + full
    attach_runtime_program(cg, b"sd_devices", ((1, 3),))              # null only
    assert probe_access(cg, paths) == "100"          # both must allow
    be = V2BpfBackend(bpffs)
    be.apply(cg, [ZERO], [], [ZERO])
    assert _names(cg) == ["gm_devallow", "gm_devallow"]
    assert probe_access(cg, paths) == "110"          # /dev/full still vetoed by "systemd"
    assert (ZERO.major, ZERO.minor) in be.allowed(cg)
    assert len([f for f in os.listdir(bpffs) if f.startswith("gm_")]) == 2
    # systemd re-realises the unit (daemon-reload) and attaches a fresh program of its own
    attach_runtime_program(cg, b"sd_devices", ((1, 3),))
    assert probe_access(cg, paths) == "100"
    assert (ZERO.major, ZERO.minor) not in be.allowed(cg)   # audit sees the veto
    be.apply(cg, [], [], [ZERO])                     # reconciler re-install
    assert _names(cg) == ["gm_devallow"] * 3
    assert probe_access(cg, paths) == "110"
    be.apply(cg, [], [ZERO], [])                     # last GPU gone: originals back, pins gone
    assert _names(cg) == ["runc_devices", "sd_devices", "sd_devices"]
    assert probe_access(cg, paths) == "100"
    assert not [f for f in os.listdir(bpffs) if f.startswith("gm_")]


def test_systemd_reload_keeps_hot_mounted_device_via_device_allow(cgroup2_child, bpffs, tmp_path):
    """A fake systemd that, like the real one, realises the unit's DeviceAllow= as a fresh device
    program on every change (ALLOW_MULTI; its previous program it tries to detach is already
    wrapped by ours). With DeviceAllow= kept in step the hot-mounted device survives it, and the
    audit accepts systemd's program because it evaluates it."""
    from gpumounter_amd.fakes.systemd_bus import FakeSystemd
    from gpumounter_amd.node.systemd import DeviceAllowSync, SystemdBus, SystemdPersistingBackend

    cg = cgroup2_child
    paths = [NULL.path, ZERO.path, FULL.path]
    unit = "cri-containerd-" + os.path.basename(cg) + ".scope"
    scope = os.path.join(os.path.dirname(cg), unit)
    os.mkdir(scope)
    try:
        def realise(_unit, entries):
            nodes = []
            for p, _perm in entries:
                st = os.stat(p)
                nodes.append((os.major(st.st_rdev), os.minor(st.st_rdev)))
            attach_runtime_program(scope, b"sd_devices", tuple(nodes))

        fs = FakeSystemd(str(tmp_path / "private"), on_change=realise).start()
        fs.add_unit(unit, [(NULL.path, "rwm")])
        attach_runtime_program(scope, b"runc_devices", ((1, 3),))
        realise(unit, fs.units[unit])                 # systemd's program from the scope's start
        assert probe_access(scope, paths) == "100"
        be = SystemdPersistingBackend(V2BpfBackend(bpffs),
                                      DeviceAllowSync(SystemdBus(fs.path), retry_s=0.01))
        be.apply(scope, [ZERO], [], [ZERO])
        assert probe_access(scope, paths) == "110"    # effective at once (BPF, request path)
        assert be.sync.flush()                        # DeviceAllow= follows; systemd re-realises
        assert fs.units[unit] == [(NULL.path, "rwm"), (ZERO.path, "rw")]
        assert _names(scope).count("sd_devices") == 1  # its new program, next to our wrappers
        assert probe_access(scope, paths) == "110"    # …which grants /dev/zero too
        assert (ZERO.major, ZERO.minor) in be.allowed(scope)
        be.apply(scope, [], [ZERO], [])               # detach: DeviceAllow= shrinks back
        assert be.sync.flush()
        assert fs.units[unit] == [(NULL.path, "rwm")]
        assert probe_access(scope, paths) == "100"
        be.sync.stop()
        fs.stop()
    finally:
        os.rmdir(scope)


def test_cgroup_v2_chain_lost_falls_back_to_oci_defaults(cgroup2_child):
    """Unpinned map + 'worker restart' (kept fd dropped): reinstall compiles in the OCI defaults."""
    cg = cgroup2_child
    attach_runtime_program(cg)
    be = V2BpfBackend("")
    be.apply(cg, [ZERO], [], [ZERO])
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "110"
    # simulate the worker process dying: close every kept map fd → the kernel empties the slot
    import gc
    lib = _native.host()
    ino = os.stat(cg).st_ino
    # the C++ registry holds one dup'd fd; find and close it via /proc/self/fd of bpf-map type
    for fd in os.listdir("/proc/self/fd"):
        try:
            if os.readlink(f"/proc/self/fd/{fd}") == "anon_inode:bpf-map":
                os.close(int(fd))
        except OSError:
            pass
    gc.collect()
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "010"  # chain broken
    be.apply(cg, [ZERO], [], [ZERO])                 # reconcile re-install: OCI defaults inline
    # the OCI default list allows /dev/null, /dev/zero and /dev/full (1:3, 1:5, 1:7)
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "111"
    assert ino


def test_cgroup_v1_devices_controller():
    base = "/sys/fs/cgroup/devices"
    if not os.path.isdir(base):
        pytest.skip("no v1 devices controller")
    cg = os.path.join(base, "gm-test-" + uuid.uuid4().hex[:8])
    os.mkdir(cg)
    try:
        with open(os.path.join(cg, "devices.deny"), "w") as fh:
            fh.write("a")
        with open(os.path.join(cg, "devices.allow"), "w") as fh:
            fh.write("c 1:3 rwm")
        paths = [NULL.path, ZERO.path]
        assert probe_access(cg, paths) == "10"
        be = V1Backend()
        be.apply(cg, [ZERO], [], [ZERO])
        assert probe_access(cg, paths) == "11"
        assert (1, 5) in be.allowed(cg)
        be.apply(cg, [], [ZERO], [])
        assert probe_access(cg, paths) == "10"
    finally:
        with open(os.path.join(cg, "cgroup.procs")) as fh:
            for pid in fh.read().split():
                with open(os.path.join(base, "cgroup.procs"), "w") as out:
                    out.write(pid)
        os.rmdir(cg)


def test_devnodes_real_mknod_via_setns(tmp_path):
    """procroot + setns modes against a real process in a private mount namespace."""
    root = tmp_path / "ctr"
    (root / "dev").mkdir(parents=True)
    # a sleeper in a new mount namespace whose /dev is a private tmpfs
    child = subprocess.Popen(["unshare", "-m", "--propagation", "private", "sh", "-c",
                              f"mount -t tmpfs tmpfs {root}/dev && echo ok && sleep 60"],
                             stdout=subprocess.PIPE, text=True)
    try:
        assert child.stdout.readline().strip() == "ok"
        from gpumounter_amd.node.devnodes import DevNodeWriter, Target

        # the node created through the child's mount namespace must be invisible from ours
        w = DevNodeWriter("setns")
        node = DeviceNode(f"{root}/dev/dri/renderD128", 226, 128)
        assert w.create(Target(pid=child.pid), [node]) == [0]
        assert not os.path.exists(f"{root}/dev/dri/renderD128")
        assert w.present(Target(pid=child.pid), node)
        w2 = DevNodeWriter("procroot")
        assert w2.present(Target(pid=child.pid), node)
        assert w2.remove(Target(pid=child.pid), [node]) == [0]
        assert not w.present(Target(pid=child.pid), node)
    finally:
        child.kill()
        child.wait()


def test_cgroup_v2_set_mode_updates_without_reloading(cgroup2_child, bpffs, monkeypatch):
    """Set mode: the first install wraps the runtime's program once; later grants and revokes
    are updates of the allow-set map (same program id, no load, no attach) that the kernel
    enforces at once. allowed() reads the set back from the kernel (no xlated interpretation);
    a foreign program joining (systemd re-realising the unit) is still evaluated."""
    from gpumounter_amd.node import cgroup as cgmod

    cg = cgroup2_child
    attach_runtime_program(cg)
    be = V2BpfBackend(bpffs)
    lib = _native.host()
    be.apply(cg, [ZERO], [], [ZERO])
    ids = be.attached_ids(cg)
    tm = _native.BpfTiming()
    lib.gm_bpf_dev_last_timing(C.byref(tm))
    assert tm.programs == 1 and probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "110"
    be.apply(cg, [FULL], [], [ZERO, FULL])
    lib.gm_bpf_dev_last_timing(C.byref(tm))
    assert tm.programs == 0 and be.attached_ids(cg) == ids     # a map update only
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "111"
    interp = []
    slow = cgmod.program_allows
    monkeypatch.setattr(cgmod, "program_allows", lambda p: interp.append(1) or slow(p))
    assert be.allowed(cg) == {(ZERO.major, ZERO.minor), (FULL.major, FULL.minor)}
    assert interp == []                                      # read from the map
    be.apply(cg, [], [FULL], [ZERO])
    assert be.attached_ids(cg) == ids and be.allowed(cg) == {(ZERO.major, ZERO.minor)}
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "110"
    # a foreign program joins: only /dev/null, so it vetoes ZERO
    attach_runtime_program(cg, name=b"sd_devices")
    assert (ZERO.major, ZERO.minor) not in be.allowed(cg)
    assert probe_access(cg, [NULL.path, ZERO.path]) == "10"
    # the re-install wraps the newcomer too, sharing the one allow set
    be.apply(cg, [], [], [ZERO])
    assert be.allowed(cg) == {(ZERO.major, ZERO.minor)}
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "110"


def test_pinned_chain_maps_of_removed_cgroups_are_swept(cgroup2_child, bpffs):
    """A container that exits while holding hot-mounted GPUs leaves its cgroup's pinned chain
    map behind (it would keep the runtime's program loaded); the reconciler's sweep unpins it
    and keeps the pins of live cgroups."""
    root = os.path.dirname(cgroup2_child)
    live, dead = cgroup2_child, os.path.join(root, "gm-dead-" + uuid.uuid4().hex[:8])
    os.mkdir(dead)
    be = V2BpfBackend(bpffs)
    for cg in (live, dead):
        attach_runtime_program(cg)
        be.apply(cg, [ZERO], [], [ZERO])
    ino_live, ino_dead = os.stat(live).st_ino, os.stat(dead).st_ino
    pins = sorted(f for f in os.listdir(bpffs) if f.startswith("gm_"))
    assert sorted(p.split("_")[1] for p in pins) == sorted([str(ino_live), str(ino_dead)])
    os.rmdir(dead)                        # the container exited: its cgroup is gone
    removed = be.sweep_pins(root)
    assert [p.split("_")[1] for p in removed] == [str(ino_dead)]
    assert [p.split("_")[1] for p in os.listdir(bpffs) if p.startswith("gm_")] == [str(ino_live)]
    assert be.sweep_pins(root) == []
    assert probe_access(live, [NULL.path, ZERO.path]) == "11"      # the live chain still works


def test_straight_line_program_upgrades_to_set_mode(cgroup2_child, bpffs):
    """GM_BPF_SET_MODE=false compiles straight-line programs (what older workers attached); a
    set-mode worker meeting one replaces it by a set-mode wrapper around the same runtime
    program, and the grants survive the swap."""
    from gpumounter_amd.node.cgroup import _set_at

    cg = cgroup2_child
    attach_runtime_program(cg)
    old = V2BpfBackend(bpffs, set_mode=False)
    old.apply(cg, [ZERO], [], [ZERO])
    assert _set_at(cg, 0) == ("code", None)
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "110"
    new = V2BpfBackend(bpffs, set_mode=True)
    new.apply(cg, [FULL], [], [ZERO, FULL])
    kind, pairs = _set_at(cg, 0)
    assert kind == "set" and pairs == {(ZERO.major, ZERO.minor), (FULL.major, FULL.minor)}
    assert len(new.attached_ids(cg)) == 1                   # replaced, not stacked
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "111"
    new.apply(cg, [], [ZERO, FULL], [])
    assert probe_access(cg, [NULL.path, ZERO.path, FULL.path]) == "100"
