"""What a process inside the tenant container sees of the GPUs.

BASELINE config "attach 1 MI355X to a running rocm/pytorch Pod; rocm-smi inside the Pod sees
it" needs a process *in the tenant's view of the node* — its own ``/dev`` and device cgroup.
On a privileged host that view is real (tests/test_privileged_e2e.py opens the injected nodes
from inside a tenant mount namespace). The GPU box allows neither namespaces nor cgroup writes,
so the worker emulates its node operations there (marker files for nodes, a recorded cgroup-v2
allow set); ``libgm_tenant_view.so`` (native/src/gm_tenant_view.cpp), preloaded into a child
process, makes that child's ROCm stack open ``/dev/kfd`` and ``/dev/dri/*`` through exactly that
emulated state. The child then reports what HIP enumerates: no GPU before an attach, the
attached GPU(s) after it, none again after the detach.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from typing import Dict, List

from gpumounter_amd import _native

_CHILD = r"""
import json, sys
sys.path.insert(0, %(root)r)
from gpumounter_amd import _native
import ctypes as C
lib = _native.probe()
n = C.c_int(0)
rc = lib.gm_probe_device_count(C.byref(n))
bdfs = []
for i in range(n.value if rc == 0 else 0):
    p = _native.ProbeProps()
    if lib.gm_probe_props(i, C.byref(p)) == 0:
        bdfs.append(p.pci_bus_id.decode().lower())
print(json.dumps({"rc": rc, "count": n.value if rc == 0 else 0, "bdfs": bdfs}))
"""


# "a running rocm/pytorch Pod": a fresh PyTorch process in the tenant's view, as a workload in
# the Pod would start after an attach. It reports what torch enumerates and, given a GPU, runs a
# bf16 GEMM on it and checks it against an fp32 host reference.
#
# The count is the HIP runtime's (``is_available()`` asks it too): what the process can open.
# On ROCm builds ``torch.cuda.device_count()`` is answered by amd-smi before CUDA-side init, and
# amd-smi enumerates from sysfs, which a container sees node-wide — it reports the node's GPUs
# whether or not this process can reach them (``device_count_api`` below; the same holds for
# ``amd-smi list`` / ``rocm-smi`` in a real container, profiles/r3_tenant_view/smi_probe.txt).
_TORCH_CHILD = r"""
import json, torch
n = torch._C._cuda_getDeviceCount() if torch.cuda.is_available() else 0
out = {"count": n, "bdfs": [], "device_count_api": torch.cuda.device_count()}
for i in range(n):
    p = torch.cuda.get_device_properties(i)
    out["bdfs"].append("%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id))
    out["arch"] = p.gcnArchName
if n:
    g = torch.Generator().manual_seed(0)
    a = torch.randn(2048, 2048, generator=g)
    b = torch.randn(2048, 2048, generator=g)
    ref = a.bfloat16().float() @ b.bfloat16().float()
    c = (a.bfloat16().cuda() @ b.bfloat16().cuda()).float().cpu()
    out["gemm_max_rel_err"] = float(((c - ref).abs().max() / ref.abs().max()).item())
print(json.dumps(out))
"""


def view_lib() -> str:
    path = _native.lib_path("libgm_tenant_view.so")
    if not os.path.exists(path):
        raise _native.NativeError(f"{path} missing — run `make -C native`")
    return path


def tenant_env(rootfs: str, cgroup_dir: str = "") -> Dict[str, str]:
    """Environment for a tenant-side child: the view library is appended to any LD_PRELOAD
    already in effect (which stays in place)."""
    env = dict(os.environ)
    pre = [p for p in env.get("LD_PRELOAD", "").split(":") if p]
    env["LD_PRELOAD"] = ":".join(pre + [view_lib()])
    env["GM_TENANT_ROOT"] = rootfs
    if cgroup_dir:
        env["GM_TENANT_CGROUP"] = cgroup_dir
    else:
        env.pop("GM_TENANT_CGROUP", None)
    return env


def hip_devices(rootfs: str, cgroup_dir: str = "", timeout: float = 120.0) -> Dict:
    """Start a fresh process in the tenant's view and return what HIP enumerates there:
    ``{"rc": hipError_t of hipGetDeviceCount, "count": n, "bdfs": [...]}``. (HIP, like CUDA,
    enumerates once per process: a running process does not see later attaches, a new one
    does — the same holds in a real container.)"""
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    res = subprocess.run([sys.executable, "-c", _CHILD % {"root": repo}],
                         env=tenant_env(rootfs, cgroup_dir), capture_output=True, text=True,
                         timeout=timeout)
    if res.returncode != 0:
        raise RuntimeError(f"tenant-side HIP check failed ({res.returncode}): "
                           f"{res.stderr[-2000:]}")
    return json.loads(res.stdout.strip().splitlines()[-1])


def torch_devices(rootfs: str, cgroup_dir: str = "", timeout: float = 300.0) -> Dict:
    """Start a fresh PyTorch process in the tenant's view: ``{"count", "bdfs", "arch",
    "gemm_max_rel_err"}`` (the GEMM only when a GPU is visible)."""
    res = subprocess.run([sys.executable, "-c", _TORCH_CHILD],
                         env=tenant_env(rootfs, cgroup_dir), capture_output=True, text=True,
                         timeout=timeout)
    if res.returncode != 0:
        raise RuntimeError(f"tenant-side PyTorch check failed ({res.returncode}): "
                           f"{res.stderr[-2000:]}")
    return json.loads(res.stdout.strip().splitlines()[-1])


def locate(rootfs_root: str, cgroup_root: str, container_id: str):
    """(rootfs dir, cgroup dir) of a fake node's container, found from the outside (the fake
    control plane may run in another process): the rootfs is ``<rootfs_root>/<id>``, the cgroup
    the directory whose marker names the container."""
    from gpumounter_amd.node.cgroup import FAKE_MARKER
    for d, _, files in os.walk(cgroup_root):
        if FAKE_MARKER in files:
            try:
                with open(os.path.join(d, FAKE_MARKER)) as fh:
                    if json.load(fh).get("container") == container_id:
                        return os.path.join(rootfs_root, container_id), d
            except (OSError, ValueError):
                continue
    raise FileNotFoundError(f"container {container_id} not under {cgroup_root}")


def check_attach_cycle(attach, detach, rootfs: str, cgroup_dir: str,
                       runtime: str = "hip") -> Dict:
    """Tenant-side view across one attach/detach: what a fresh HIP (``runtime="hip"``) or
    PyTorch (``"pytorch"``) process enumerates before, during and after. ``attach()`` returns
    the attached BDFs; ``detach()`` removes them."""
    look = torch_devices if runtime == "pytorch" else hip_devices
    before = look(rootfs, cgroup_dir)
    bdfs = sorted(b.lower() for b in attach())
    try:
        during = look(rootfs, cgroup_dir)
    finally:
        detach()
    after = look(rootfs, cgroup_dir)
    ok = before["count"] == 0 and sorted(during["bdfs"]) == bdfs and after["count"] == 0
    out = {"ok": ok, "before": before["count"], "during": during["bdfs"],
           "after": after["count"], "attached": bdfs,
           "how": f"fresh {'PyTorch' if runtime == 'pytorch' else 'HIP'} process; /dev/kfd, "
                  "/dev/dri/* and the device-cgroup verdict resolved through the emulated node "
                  "state (libgm_tenant_view.so)"}
    if runtime == "pytorch":
        ok = ok and during.get("gemm_max_rel_err", 1.0) < 1e-2
        out.update(ok=ok, gemm_max_rel_err=during.get("gemm_max_rel_err"),
                   arch=during.get("arch"), device_count_api=during.get("device_count_api"))
    return out


def can_open(rootfs: str, paths: List[str], cgroup_dir: str = "") -> Dict[str, int]:
    """errno of ``open(path, O_RDWR)`` for each path in the tenant's view (0 = opened)."""
    code = ("import errno, json, os, sys\n"
            "out = {}\n"
            "for p in sys.argv[1:]:\n"
            "    try:\n"
            "        os.close(os.open(p, os.O_RDWR | os.O_CLOEXEC)); out[p] = 0\n"
            "    except OSError as e:\n"
            "        out[p] = e.errno\n"
            "print(json.dumps(out))\n")
    res = subprocess.run([sys.executable, "-c", code, *paths],
                         env=tenant_env(rootfs, cgroup_dir), capture_output=True, text=True,
                         timeout=60)
    if res.returncode != 0:
        raise RuntimeError(res.stderr[-2000:])
    return json.loads(res.stdout.strip().splitlines()[-1])
