"""Driver for tests/test_privileged_userns.py (root; run under `unshare -m --propagation private`
so the staging tmpfs it mounts dies with it).

A tenant in its own **user** and mount namespace mounts a tmpfs on its /dev from inside that
user namespace, as a container runtime does for a Kubernetes `hostUsers: false` pod. The kernel
treats that tmpfs as nodev. Checked, with /dev/null's numbers (1:3) standing in for a GPU node:
  * mknod mode (the reference's method) creates a node the tenant cannot open;
  * bind mode (auto-detected from the tenant's user namespace) gives a node it can open, owned
    by its root, invisible from the worker's namespace, replacing the unusable mknod'ed one;
  * create is idempotent, the read-back requires the mount, removal unmounts and unlinks.
Prints one JSON line.
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpumounter_amd import _native  # noqa: E402
from gpumounter_amd.models.device import DeviceNode  # noqa: E402
from gpumounter_amd.node.devnodes import DevNodeWriter, Target  # noqa: E402


def tenant_can_open(pid: int, path: str) -> bool:
    r = subprocess.run(["nsenter", "-t", str(pid), "-U", "-m", "sh", "-c",
                        ': <> "$1" 2>/dev/null && echo 1 || echo 0', "sh", path],
                       capture_output=True, text=True, timeout=30)
    return r.stdout.strip() == "1"


def tenant_ls(pid: int, path: str) -> str:
    r = subprocess.run(["nsenter", "-t", str(pid), "-U", "-m", "stat", "-c", "%F %t:%T %a %u",
                        path], capture_output=True, text=True, timeout=30)
    return r.stdout.strip() if r.returncode == 0 else ""


def main() -> int:
    base = tempfile.mkdtemp(prefix="gm-userns-")
    root = os.path.join(base, "ctr")
    os.makedirs(os.path.join(root, "dev"))
    stage = os.path.join(base, "run", "gpumounter", "devstage")   # parents created on demand
    tenant = subprocess.Popen(
        ["unshare", "-U", "--map-user=0", "--map-group=0", "-m", "--propagation", "private",
         "sh", "-c", f"mount -t tmpfs tmpfs {root}/dev && echo ok && exec sleep 120"],
        stdout=subprocess.PIPE, text=True)
    out = {}
    try:
        assert tenant.stdout.readline().strip() == "ok", "tenant setup failed"
        t = Target(pid=tenant.pid)
        node = DeviceNode(f"{root}/dev/dri/renderD128", 1, 3)

        # the reference's method: the node exists, passes a plain read-back, cannot be opened
        mk = DevNodeWriter("setns", userns="off")
        out["mknod_result"] = mk.create(t, [node])
        out["mknod_present"] = mk.present_many(t, [node])
        out["mknod_tenant_open"] = tenant_can_open(tenant.pid, node.path)

        w = DevNodeWriter("procroot", userns="auto", stage_dir=stage)
        out["bind_detected"] = w._bind(t)
        out["bind_present_before"] = w.present_many(t, [node])   # mknod'ed node does not count
        out["bind_create"] = w.create(t, [node])                 # replaces it
        out["bind_tenant_open"] = tenant_can_open(tenant.pid, node.path)
        out["bind_tenant_stat"] = tenant_ls(tenant.pid, node.path)
        out["bind_invisible_here"] = not os.path.exists(node.path)
        out["bind_present"] = w.present_many(t, [node])
        out["bind_create_again"] = w.create(t, [node])
        kfd = DeviceNode(f"{root}/dev/kfd", 1, 3)
        out["bind_second_node"] = w.create(t, [kfd])
        out["bind_remove"] = w.remove(t, [node, kfd])
        out["after_remove_stat"] = tenant_ls(tenant.pid, node.path)
        out["after_remove_present"] = w.present_many(t, [node])
        out["remove_again"] = w.remove(t, [node])
        # a mknod-mode writer meeting a bind-mounted node unmounts it through the namespace
        w.create(t, [node])
        plain = DevNodeWriter("procroot", userns="off", stage_dir=stage)
        out["plain_remove_of_bound"] = plain.remove(t, [node])
        out["plain_after"] = tenant_ls(tenant.pid, node.path)
    finally:
        tenant.kill()
        tenant.wait()
        _native.host().gm_devnodes_stage(None, 0)
        subprocess.run(["umount", "-l", stage], check=False)
        shutil.rmtree(base, ignore_errors=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
