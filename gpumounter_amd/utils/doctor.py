"""Node preflight: ``python -m gpumounter_amd doctor`` checks everything the worker needs on a node.

The reference has no such tool; its failure modes surface as a failed attach (wrong cgroup driver
env, missing ``mknod`` in the image, no kubelet socket — reference docs/guide/FAQ.md:3-7). Each
check here reports ``ok``, ``warn`` (works, but a feature is degraded) or ``fail`` (attaches
cannot work), with the detail an operator needs. Run it in the worker container (same mounts and
privileges as the DaemonSet) or on the host with the same ``GM_*`` settings.
"""
from __future__ import annotations

import asyncio
import ctypes as C
import errno
import json
import os
from dataclasses import asdict, dataclass
from typing import List

from gpumounter_amd import _native

BPF_FS_MAGIC = 0xCAFE4A11


@dataclass
class Check:
    name: str
    status: str          # ok | warn | fail
    detail: str


def _statfs_type(path: str) -> int:
    class StatFs(C.Structure):
        _fields_ = [("f_type", C.c_long), ("rest", C.c_byte * 120)]

    libc = C.CDLL(None, use_errno=True)
    buf = StatFs()
    if libc.statfs(path.encode(), C.byref(buf)) != 0:
        raise OSError(C.get_errno(), os.strerror(C.get_errno()), path)
    return buf.f_type & 0xFFFFFFFF


def check_inventory(cfg) -> List[Check]:
    from gpumounter_amd.hw.inventory import Inventory

    try:
        inv = Inventory(cfg.amdsmi_lib, cfg.kfd_major, cfg.kfd_dev_path)
        gpus = inv.gpus()
    except Exception as e:  # noqa: BLE001
        return [Check("amdsmi", "fail", f"inventory unavailable: {e}")]
    out = [Check("amdsmi", "ok" if gpus else "fail",
                 f"{len(gpus)} GPU(s) via {inv.lib_path}: "
                 + ", ".join(sorted({g.gfx_target for g in gpus})))]
    hives = {g.xgmi_hive_id for g in gpus}
    out.append(Check("xgmi", "ok" if len(gpus) < 2 or len(hives) == 1 else "warn",
                     f"{len(hives)} hive(s) for {len(gpus)} GPU(s)"))
    kfd_src = "configured" if cfg.kfd_major else (
        cfg.kfd_dev_path if os.path.exists(cfg.kfd_dev_path) else "fallback 511")
    out.append(Check("kfd", "ok" if kfd_src != "fallback 511" else "warn",
                     f"/dev/kfd major {inv.kfd_major} ({kfd_src})"))
    return out


def check_cgroup(cfg) -> List[Check]:
    from gpumounter_amd.node.cgroup import CgroupResolver

    root = cfg.cgroup_root
    if not os.path.isdir(root):
        return [Check("cgroup", "fail", f"{root} is not mounted")]
    mode = CgroupResolver.detect_mode(root) if cfg.cgroup_mode == "auto" else cfg.cgroup_mode
    out = []
    if mode == "v1":
        allow = os.path.join(root, "devices", "devices.allow")
        ok = os.access(allow, os.W_OK)
        out.append(Check("cgroup", "ok" if ok else "fail",
                         f"v1 devices controller, {allow} {'writable' if ok else 'NOT writable'}"))
        return out
    out.append(Check("cgroup", "ok", f"v2 unified hierarchy at {root}"))
    # can this process load a device program? (CAP_BPF + CAP_SYS_ADMIN in the DaemonSet)
    from gpumounter_amd.node.cgroup import _rule_array, rules_for
    from gpumounter_amd.models.device import DeviceNode

    lib = _native.host()
    rules = rules_for([DeviceNode("/dev/null", 1, 3)], allow=True)
    need = -lib.gm_bpf_dev_build(_rule_array(rules), 1, 0, -1, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build(_rule_array(rules), 1, 0, -1, buf, need)
    fd = lib.gm_bpf_dev_load(buf, n, b"gm_doctor", None, 0)
    if fd >= 0:
        os.close(fd)
        out.append(Check("bpf", "ok", "BPF_PROG_TYPE_CGROUP_DEVICE programs load"))
    else:
        out.append(Check("bpf", "fail", f"cannot load a device program: {os.strerror(-fd)} "
                                        "(needs CAP_BPF/CAP_SYS_ADMIN: privileged DaemonSet)"))
    if fd >= 0 and cfg.bpf_set_mode:
        rc = lib.gm_bpf_dev_probe_set()
        out.append(Check("bpf-set", "ok" if rc == 0 else "warn",
                         "allow-set programs load (grants are map updates)" if rc == 0 else
                         f"allow-set program refused ({os.strerror(-rc)}): set "
                         "GM_BPF_SET_MODE=false for straight-line programs"))
    pin = cfg.bpf_pin_dir
    if pin:
        parent = pin if os.path.isdir(pin) else os.path.dirname(pin)
        try:
            is_bpffs = _statfs_type(parent) == BPF_FS_MAGIC
        except OSError as e:
            is_bpffs = False
            parent = f"{parent} ({e.strerror})"
        out.append(Check("bpffs", "ok" if is_bpffs else "warn",
                         f"{parent} is {'a' if is_bpffs else 'not a'} bpffs: tail-call maps "
                         + ("survive worker restarts" if is_bpffs else
                            "are kept in-process only (lost on restart until reconciled)")))
    return out


def check_devnodes(cfg) -> List[Check]:
    """User-namespaced Pods (hostUsers: false) get bind-mounted nodes (open_tree + move_mount,
    node/devnodes.py), which needs CAP_SYS_ADMIN and a ≥5.2 kernel."""
    if cfg.devnode_userns == "off" or cfg.devnode_mode == "emulate":
        return [Check("devnodes-userns", "ok", f"bind mode not used (devnode_userns="
                                               f"{cfg.devnode_userns}, mode={cfg.devnode_mode})")]
    rc = _native.host().gm_devnodes_bind_probe()
    if rc == 0:
        return [Check("devnodes-userns", "ok", "open_tree/move_mount available: user-namespaced "
                                               "Pods get bind-mounted device nodes")]
    return [Check("devnodes-userns", "warn",
                  f"open_tree refused ({os.strerror(-rc)}): attaches to user-namespaced Pods "
                  "(hostUsers: false) will fail; other Pods are unaffected")]


def check_pidns(cfg) -> List[Check]:
    """Busy detection's process tables (KFD's and amdsmi's) name host-namespace PIDs
    (``profiles/r6_kfd_probe/``); the worker uses them only in the host PID namespace."""
    from gpumounter_amd.node import procs

    host = procs.host_pid_ns()
    table = ""
    if cfg.kfd_proc_path:
        try:
            n = len({p for t in procs.kfd_table(cfg.kfd_proc_path).values() for p in t})
            table = f"; KFD process table readable ({n} process(es) on a GPU)"
        except OSError as e:
            table = f"; KFD process table {cfg.kfd_proc_path}: {e.strerror} (amdsmi's is used)"
    if host:
        return [Check("pidns", "ok", "host PID namespace (hostPID): busy detection can use the "
                                     "KFD/amdsmi process tables" + table)]
    return [Check("pidns", "warn",
                  "not in the host PID namespace: busy detection relies on the render-fd scan "
                  "alone (the KFD/amdsmi tables name host PIDs); run the DaemonSet with "
                  "hostPID: true" + table)]


def check_systemd(cfg) -> List[Check]:
    from gpumounter_amd.node import systemd

    if cfg.systemd_device_allow == "off":
        return [Check("systemd", "ok", "DeviceAllow persistence disabled")]
    bus = systemd.find_bus(cfg.systemd_bus)
    if bus is None:
        status = "fail" if cfg.systemd_device_allow == "on" else (
            "warn" if cfg.cgroup_driver == "systemd" else "ok")
        detail = ("no systemd bus socket mounted (/run/systemd or /run/dbus): on "
                  "systemd-driver nodes a daemon-reload can drop hot-mounted devices until the "
                  "reconciler restores them") if status != "ok" else \
            "no systemd bus socket (needed only with the systemd cgroup driver)"
        return [Check("systemd", status, detail)]
    err = C.create_string_buffer(256)
    out = C.create_string_buffer(1 << 12)
    rc = _native.host().gm_sd_get_device_allow(bus.encode(), b"-.slice", out, 1 << 12, err, 256)
    if rc >= 0 or rc == -errno.EPROTO:   # a D-Bus answer (even an error) means we are talking
        return [Check("systemd", "ok", f"systemd reachable on {bus}")]
    return [Check("systemd", "warn", f"{bus}: {err.value.decode() or os.strerror(-rc)}")]


async def _check_dra(cfg) -> List[Check]:
    """gpu_allocation=dra: the node's ResourceSlice must publish its GPUs with a PCI address
    the worker can map to amdsmi's inventory."""
    from gpumounter_amd.cluster.kube import KubeClient
    from gpumounter_amd.hw.inventory import Inventory
    from gpumounter_amd.models.device import normalize_device_id
    from gpumounter_amd.node.dra import DraLedger

    try:
        kube = KubeClient.from_config(cfg)
    except Exception as e:  # noqa: BLE001
        return [Check("dra", "fail", f"no credentials: {e}")]
    led = DraLedger(kube, cfg.node_name, cfg.dra_driver, cfg.dra_device_class,
                    cfg.dra_bdf_attribute)
    try:
        devs = await led.allocatable()
        allocs = await led.list()
    except Exception as e:  # noqa: BLE001
        return [Check("dra", "fail", f"resource.k8s.io/v1: {e}")]
    finally:
        await kube.close()
    if not devs:
        return [Check("dra", "fail", f"no ResourceSlice device of driver {cfg.dra_driver} on "
                                     f"{cfg.node_name} carries a PCI address "
                                     f"(attribute {cfg.dra_bdf_attribute!r})")]
    try:
        have = {normalize_device_id(g.bdf) for g in Inventory(
            cfg.amdsmi_lib, cfg.kfd_major, cfg.kfd_dev_path).gpus()}
    except Exception:  # noqa: BLE001 - reported by the amdsmi check
        have = set()
    unknown = [d for d in devs if have and normalize_device_id(d) not in have]
    if unknown:
        return [Check("dra", "warn", f"ResourceSlice devices not in the amdsmi inventory: "
                                     f"{unknown}")]
    return [Check("dra", "ok", f"{len(devs)} {cfg.dra_driver} device(s) in ResourceSlices, "
                               f"{len(allocs)} claim reservation(s) on this node")]


async def _check_kubelet(cfg) -> List[Check]:
    from gpumounter_amd.node.ledger import LedgerClient

    if getattr(cfg, "gpu_allocation", "device-plugin") == "dra":
        return await _check_dra(cfg)
    if not os.path.exists(cfg.kubelet_socket):
        return [Check("kubelet", "fail", f"PodResources socket {cfg.kubelet_socket} missing")]
    lc = LedgerClient(cfg.kubelet_socket, cfg.resource_name, cfg.kubelet_timeout_s,
                      cfg.podresources_api)
    try:
        allocs = await lc.list()
        alloc = await lc.allocatable()
        return [Check("kubelet", "ok",
                      f"PodResources {lc.api_version}: {len(allocs)} {cfg.resource_name} "
                      f"allocation(s)" + (f", {len(alloc)} allocatable" if alloc else ""))]
    except Exception as e:  # noqa: BLE001
        return [Check("kubelet", "fail", f"PodResources List failed: {e}")]
    finally:
        await lc.close()


async def _check_apiserver(cfg) -> List[Check]:
    from gpumounter_amd.cluster.kube import KubeClient

    try:
        kube = KubeClient.from_config(cfg)
    except Exception as e:  # noqa: BLE001
        return [Check("apiserver", "fail", f"no credentials: {e}")]
    try:
        pods, _ = await kube.list_pods(cfg.pool_namespace)
        out = [Check("apiserver", "ok", f"{kube.base}: {len(pods)} pod(s) in "
                                        f"{cfg.pool_namespace}")]
    except Exception as e:  # noqa: BLE001
        await kube.close()
        return [Check("apiserver", "fail", f"{kube.base}: {e}")]
    try:
        return out + await _check_priority(cfg, kube)
    finally:
        await kube.close()


async def _check_priority(cfg, kube) -> List[Check]:
    """The placeholders' floor PriorityClass exists (and the pool's, when one is set). Without
    it placeholders rank as their tenants do, and a higher-priority Pod can preempt a
    placeholder — revoking a GPU a tenant is using."""
    from gpumounter_amd.cluster.kube import NotFound

    out = []
    for what, name in (("placeholder", cfg.placeholder_priority_class),
                       ("pool", getattr(cfg, "pool_priority_class", ""))):
        if not name:
            if what == "placeholder":
                out.append(Check("priority", "warn", "no placeholder_priority_class: "
                                 "placeholders rank as their tenants"))
            continue
        try:
            pc = await kube.get_priority_class(name)
        except NotFound:
            out.append(Check("priority", "fail", f"{what} PriorityClass {name} missing "
                                                 f"(kubectl apply -f deploy/placeholder-"
                                                 f"priority.yaml)"))
            continue
        except Exception as e:  # noqa: BLE001
            out.append(Check("priority", "warn", f"{what} PriorityClass {name}: {e}"))
            continue
        out.append(Check("priority", "ok", f"{what} PriorityClass {name}: value "
                                           f"{pc.get('value')}, preemptionPolicy "
                                           f"{pc.get('preemptionPolicy', 'PreemptLowerPriority')}"))
    return out


def check_gpus(cfg, burn_in_s: float = 0.0) -> List[Check]:
    """Run the gfx950 probe kernels on every GPU of the node (``doctor --gpu``): each amdsmi GPU
    must be visible to HIP and pass the wave64 liveness kernel. With ``burn_in_s`` also a
    sustained bit-checked bf16 GEMM load per GPU. A GPU that fails here should not be handed
    out."""
    from gpumounter_amd.hw.inventory import Inventory
    from gpumounter_amd.ops import probe

    try:
        n = probe.device_count()
    except Exception as e:  # noqa: BLE001 - no HIP runtime / driver
        return [Check("gpu", "fail", f"HIP unavailable: {e}")]
    if n == 0:
        return [Check("gpu", "fail", "no GPU visible to HIP")]
    try:
        want = [g.bdf for g in Inventory(cfg.amdsmi_lib, cfg.kfd_major,
                                         cfg.kfd_dev_path).gpus()]
    except Exception:  # noqa: BLE001 - reported by the amdsmi check
        want = []
    out: List[Check] = []
    seen = set()
    for d in range(n):
        try:
            pr = probe.props(d)
            seen.add(pr["pci_bus_id"])
            cold = probe.quick(d)          # includes loading the code object
            us = probe.quick(d)
            arch = pr["gcn_arch"].split(":")[0]
            detail = (f"{pr['pci_bus_id']} {arch}: liveness kernel {us:.0f} µs "
                      f"(first launch {cold / 1e3:.0f} ms)")
            status = "ok" if arch == "gfx950" else "warn"
            if burn_in_s > 0:
                b = probe.burn_in(d, burn_in_s)
                detail += (f", burn-in {b['seconds']:g} s {b['tflops']:.0f} TF/s "
                           f"{b['mismatches']} mismatching words")
                status = status if b["ok"] else "fail"
            out.append(Check(f"gpu{d}", status, detail))
        except Exception as e:  # noqa: BLE001 - a faulting GPU is exactly what this finds
            out.append(Check(f"gpu{d}", "fail", f"probe failed: {e}"))
    missing = [b for b in want if b.lower() not in seen]
    if missing:
        out.append(Check("gpu", "warn", f"amdsmi GPUs not visible to HIP here: {missing}"))
    return out


def run(cfg, skip_cluster: bool = False, gpu: bool = False,
        burn_in_s: float = 0.0) -> List[Check]:
    checks = check_inventory(cfg) + check_cgroup(cfg) + check_devnodes(cfg) + \
        check_pidns(cfg) + check_systemd(cfg)
    if gpu:
        checks += check_gpus(cfg, burn_in_s)
    if not skip_cluster:
        async def both():
            return await _check_kubelet(cfg) + await _check_apiserver(cfg)
        checks += asyncio.run(both())
    checks.append(Check("roctx", "ok" if _native.host().gm_roctx_available() else "warn",
                        "rocprofiler roctx markers " + (
                            "available" if _native.host().gm_roctx_available()
                            else "unavailable (attach/detach ranges not traced)")))
    return checks


def render(checks: List[Check], as_json: bool = False) -> str:
    if as_json:
        return json.dumps([asdict(c) for c in checks], indent=1)
    w = max(len(c.name) for c in checks)
    return "\n".join(f"{c.status.upper():4}  {c.name:<{w}}  {c.detail}" for c in checks)
