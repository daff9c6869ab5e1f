"""Full-stack attach/detach on a real kernel (run by tests/test_privileged_e2e.py as root).

HTTP master → gRPC worker → placeholder ledger (fake apiserver/kubelet) → the production node
path: real cgroup2 hierarchy, real BPF_PROG_TYPE_CGROUP_DEVICE program swapped over a
runc-style program, real mknod through /proc/<pid>/root into a tenant process that lives in its
own mount namespace (private tmpfs /dev), and — for a tenant in its own user namespace as well
(Kubernetes `hostUsers: false`), whose /dev tmpfs is nodev — real bind mounts of staged nodes
(open_tree + move_mount). The mock inventory maps the "GPUs" to harmless memory
devices (render/card minors of major 1) so a process inside the tenant cgroup can prove what the
kernel enforces. Prints one JSON line of observations.
"""
import asyncio
import ctypes as C
import json
import os
import shutil
import stat
import subprocess
import sys
import tempfile
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpumounter_amd import _native  # noqa: E402
from gpumounter_amd.fakes.harness import LocalCluster  # noqa: E402
from gpumounter_amd.fakes.realnode import attach_runtime_program  # noqa: E402
from gpumounter_amd.utils import log  # noqa: E402

PATHS = ["/dev/null", "/dev/zero", "/dev/full", "/dev/random"]
PROBE = ("import os,sys\n"
         "open(sys.argv[1]+'/cgroup.procs','w').write(str(os.getpid()))\n"
         "out=[]\n"
         "for p in sys.argv[2:]:\n"
         "    try:\n"
         "        open(p,'rb').close(); out.append('1')\n"
         "    except OSError:\n"
         "        out.append('0')\n"
         "print(''.join(out))\n")


def probe(cg):
    r = subprocess.run([sys.executable, "-c", PROBE, cg] + PATHS, capture_output=True,
                       text=True, timeout=30)
    if r.returncode:
        raise RuntimeError(r.stderr)
    return r.stdout.strip()


def prog_names(cg):
    lib = _native.host()
    ids = (C.c_uint32 * 8)()
    n, flags = C.c_uint32(0), C.c_uint32(0)
    assert lib.gm_bpf_dev_query(cg.encode(), ids, 8, C.byref(n), C.byref(flags)) == 0
    out = []
    for i in range(n.value):
        name = C.create_string_buffer(32)
        lib.gm_bpf_prog_name(ids[i], name, 32)
        out.append(name.value.decode())
    return out


HOST_PATHS = ("/dev/kfd", "/dev/dri/renderD5", "/dev/dri/card7")


def host_dev_state():
    """The worker's own /dev entries the tenant's nodes would be named like: whether each
    exists and which inode it is (compared before and after, not assumed absent)."""
    out = {}
    for p in HOST_PATHS:
        try:
            st = os.lstat(p)
            out[p] = [st.st_ino, st.st_ctime_ns]
        except FileNotFoundError:
            out[p] = None
    return out


def chr_node(pid, rel):
    try:
        st = os.stat(f"/proc/{pid}/root{rel}")
    except FileNotFoundError:
        return None
    return [os.major(st.st_rdev), os.minor(st.st_rdev)] if stat.S_ISCHR(st.st_mode) else "notchr"


async def flow(mnt, bpffs, tenant_pid, obs, hostdev="", shared_pid=0, userns_pid=0,
               stage=""):
    async with LocalCluster(cgroup_mode="v2", devnode_mode="procroot", cgroup_root=mnt,
                            kfd_major=1,
                            worker_overrides={"drm_major": 1, "bpf_pin_dir": bpffs,
                                              "host_dev_path": hostdev,
                                              "devnode_stage_dir": stage,
                                              "device_guard_period_s": float(os.environ.get("GM_TEST_GUARD", "1.0"))}) as lc:
        w = lc.nodes["node-0"].worker
        host_before = host_dev_state()
        obs["backend"] = w.backend.name
        lc.tenant("t", pids={"main": [tenant_pid]})
        node = lc.nodes["node-0"].node
        (c,) = [c for c in node.containers.values() if c.pod_name == "t"]
        cg = c.cgroup_dir
        obs["tenant_in_cgroup"] = str(tenant_pid) in open(os.path.join(cg, "cgroup.procs")).read()
        attach_runtime_program(cg)
        obs["before"] = probe(cg)
        code, b1 = await lc.add("default", "t", 1)
        obs["add1"] = [code, [d["bdf"] for d in b1.get("devices", [])]]
        obs["after_add1"] = probe(cg)
        obs["progs_after_add1"] = prog_names(cg)
        obs["nodes_after_add1"] = {p: chr_node(tenant_pid, p) for p in
                                   ("/dev/kfd", "/dev/dri/renderD5", "/dev/dri/card7")}
        obs["host_dev_untouched"] = host_dev_state() == host_before
        obs["audit_after_add1"] = [i.kind for i in await lc.audit("default", "t")]
        code, b2 = await lc.add("default", "t", 1)
        obs["add2"] = [code, [d["bdf"] for d in b2.get("devices", [])]]
        obs["after_add2"] = probe(cg)
        code, _ = await lc.remove("default", "t", [b1["devices"][0]["uuid"]])
        obs["remove1"] = code
        obs["after_remove1"] = probe(cg)
        obs["nodes_after_remove1"] = {p: chr_node(tenant_pid, p) for p in
                                      ("/dev/kfd", "/dev/dri/renderD5", "/dev/dri/renderD8")}
        code, _ = await lc.remove("default", "t", [b2["devices"][0]["uuid"]])
        obs["remove2"] = code
        obs["after_remove2"] = probe(cg)
        obs["progs_final"] = prog_names(cg)
        obs["nodes_final"] = {p: chr_node(tenant_pid, p) for p in ("/dev/kfd",
                                                                  "/dev/dri/renderD8")}
        obs["audit_final"] = [i.kind for i in await lc.audit("default", "t")]
        obs["pins_left"] = [f for f in os.listdir(bpffs) if f.startswith("gm_")]
        await guard_flow(lc, cg, obs)
        if shared_pid:
            await shared_dev_flow(lc, hostdev, shared_pid, obs)
        if userns_pid:
            await userns_flow(lc, userns_pid, obs)
        obs["host_dev_untouched_at_end"] = host_dev_state() == host_before


async def guard_flow(lc, cg, obs):
    """The runtime attaches a fresh device program next to gpumounter's (runc update, a runtime
    re-applying its rules): under BPF_F_ALLOW_MULTI it vetoes the hot-mounted GPU until the
    worker's device guard (1 s period, the shipped default) notices and re-wraps the stack."""
    code, b = await lc.add("default", "t", 1)
    obs["guard_add"] = code
    obs["guard_before_swap"] = probe(cg)
    attach_runtime_program(cg)
    t0 = time.monotonic()
    obs["guard_right_after_swap"] = probe(cg)
    while time.monotonic() - t0 < 5.0:
        got = await asyncio.get_running_loop().run_in_executor(None, probe, cg)
        if got == obs["guard_before_swap"]:
            break
        await asyncio.sleep(0.02)
    obs["guard_restored_s"] = round(time.monotonic() - t0, 3)
    obs["guard_after"] = probe(cg)
    obs["guard_repairs"] = lc.nodes["node-0"].worker.reconciler.guard_repairs
    code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
    obs["guard_remove"] = code
    obs["guard_final"] = probe(cg)
    obs["guard_audit_final"] = [i.kind for i in await lc.audit("default", "t")]


USERNS_PROBE = ("import sys\n"
                "sys.stdin.readline()\n"          # wait until moved into the tenant's cgroup
                "out=[]\n"
                "for p in sys.argv[1:]:\n"
                "    try:\n"
                "        open(p,'rb').close(); out.append('1')\n"
                "    except OSError:\n"
                "        out.append('0')\n"
                "print(''.join(out))\n")


def probe_inside(pid, cg, paths):
    """Opens `paths` from a process inside the tenant's user + mount namespaces *and* its
    cgroup: the device nodes must exist there and be openable, and the device program allow."""
    p = subprocess.Popen(["nsenter", "-t", str(pid), "-U", "-m", sys.executable, "-c",
                          USERNS_PROBE] + paths, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    with open(os.path.join(cg, "cgroup.procs"), "w") as fh:
        fh.write(str(p.pid))
    out, err = p.communicate("go\n", timeout=30)
    if p.returncode:
        raise RuntimeError(err)
    return out.strip()


async def userns_flow(lc, pid, obs):
    lc.tenant("u", pids={"main": [pid]})
    node = lc.nodes["node-0"].node
    (c,) = [c for c in node.containers.values() if c.pod_name == "u"]
    attach_runtime_program(c.cgroup_dir)
    paths = ["/dev/dri/renderD5", "/dev/dri/card7"]
    obs["userns_before"] = probe_inside(pid, c.cgroup_dir, paths)
    code, b = await lc.add("default", "u", 1)
    obs["userns_add"] = [code, sorted(d["render_minor"] for d in b.get("devices", []))]
    obs["userns_after_add"] = probe_inside(pid, c.cgroup_dir, paths)
    obs["userns_audit"] = [i.kind for i in await lc.audit("default", "u")]
    code, _ = await lc.remove("default", "u", [d["uuid"] for d in b["devices"]])
    obs["userns_remove"] = code
    obs["userns_after_remove"] = probe_inside(pid, c.cgroup_dir, paths)
    obs["userns_nodes_final"] = {p: chr_node(pid, p) for p in paths + ["/dev/kfd"]}


def listing(d):
    out = {}
    for dp, _, files in os.walk(d):
        for f in files:
            st = os.lstat(os.path.join(dp, f))
            out[os.path.relpath(os.path.join(dp, f), d)] = [os.major(st.st_rdev),
                                                            os.minor(st.st_rdev)]
    return out


async def shared_dev_flow(lc, hostdev, pid, obs):
    """A tenant whose /dev is a bind mount of the host-like dev dir (hostPath /dev): attach,
    reconcile after its placeholder vanished, and detach must leave that directory as it was."""
    lc.tenant("shared", pids={"main": [pid]})
    obs["shared_sees_host_dev"] = chr_node(pid, "/dev/dri/renderD5") == [1, 5]
    before = listing(hostdev)
    # both GPUs: renderD8/card9 do not exist in the host dir, so only the guard keeps the
    # worker from creating them there
    code, b = await lc.add("default", "shared", 2)
    obs["shared_add"] = code
    obs["shared_gpus"] = sorted(d["render_minor"] for d in b.get("devices", []))
    obs["shared_after_add_unchanged"] = listing(hostdev) == before
    w = lc.nodes["node-0"].worker
    for ph in lc.cluster.placeholders():
        lc.cluster.delete(ph["metadata"]["namespace"], ph["metadata"]["name"], grace=0)
    await asyncio.sleep(0.1)
    rep = await w.reconciler.run_once()
    obs["shared_sweep_unlinked"] = rep.orphans
    obs["shared_after_sweep_unchanged"] = listing(hostdev) == before
    obs["shared_host_listing"] = sorted(before)


def main():
    log.setup("WARNING", json_format=False)
    obs = {}
    mnt = tempfile.mkdtemp(prefix="gm-e2e-cg2-")
    bpffs = tempfile.mkdtemp(prefix="gm-e2e-bpffs-")
    subprocess.run(["mount", "-t", "cgroup2", "none", mnt], check=True)
    subprocess.run(["mount", "-t", "bpf", "bpf", bpffs], check=True)
    root = os.path.join(mnt, "gm-e2e-" + uuid.uuid4().hex[:8])
    tenant = subprocess.Popen(
        ["unshare", "-m", "--propagation", "private", "sh", "-c",
         "set -e; mount -t tmpfs tmpfs /dev; echo ok; exec sleep 300"],
        stdout=subprocess.PIPE, text=True)
    # a host-like /dev with real nodes (the worker's host_dev_path) and a second tenant that
    # bind-mounts it at /dev, as a hostPath-/dev or privileged container does
    hostdev = tempfile.mkdtemp(prefix="gm-e2e-hostdev-")
    os.makedirs(os.path.join(hostdev, "dri"))
    for rel, mi in (("kfd", 0), ("dri/renderD5", 5), ("dri/card7", 7)):
        os.mknod(os.path.join(hostdev, rel), 0o666 | stat.S_IFCHR, os.makedev(1, mi))
    shared = subprocess.Popen(
        ["unshare", "-m", "--propagation", "private", "sh", "-c",
         f"set -e; mount --bind {hostdev} /dev; echo ok; exec sleep 300"],
        stdout=subprocess.PIPE, text=True)
    # a tenant in its own user namespace: its /dev tmpfs is mounted from inside it (nodev)
    userns = subprocess.Popen(
        ["unshare", "-U", "--map-user=0", "--map-group=0", "-m", "--propagation", "private",
         "sh", "-c", "set -e; mount -t tmpfs tmpfs /dev; echo ok; exec sleep 300"],
        stdout=subprocess.PIPE, text=True)
    stage = tempfile.mkdtemp(prefix="gm-e2e-stage-")
    try:
        assert tenant.stdout.readline().strip() == "ok"
        assert shared.stdout.readline().strip() == "ok"
        assert userns.stdout.readline().strip() == "ok"
        assert os.readlink(f"/proc/{tenant.pid}/ns/mnt") != os.readlink("/proc/self/ns/mnt")
        asyncio.run(flow(root, bpffs, tenant.pid, obs, hostdev, shared.pid, userns.pid, stage))
    finally:
        for p in (tenant, shared, userns):
            p.kill()
            p.wait()
        _native.host().gm_devnodes_stage(None, 0)
        subprocess.run(["umount", "-l", stage], check=False)
        shutil.rmtree(stage, ignore_errors=True)
        shutil.rmtree(hostdev, ignore_errors=True)
        # tear the real cgroup tree down bottom-up (processes are gone)
        for dirpath, dirs, _ in sorted(os.walk(root), key=lambda t: -t[0].count("/")):
            try:
                os.rmdir(dirpath)
            except OSError:
                pass
        subprocess.run(["umount", bpffs], check=False)
        subprocess.run(["umount", mnt], check=False)
        shutil.rmtree(bpffs, ignore_errors=True)
        os.rmdir(mnt)
    print(json.dumps(obs))


if __name__ == "__main__":
    main()
