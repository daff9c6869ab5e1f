"""A fake Kubernetes node: device-plugin ledger, container runtime artifacts, cgroupfs.

The reference tests need a live cluster, real GPUs and root (reference: pkg/util/cgroup/
cgroup_test.go:37-38 writes the real devices.allow; namespace_test.go:11 hard-codes a PID) —
SURVEY §4. This node emulates exactly the host surfaces the worker touches:

* the ``amd.com/gpu`` device plugin: capacity, device IDs (PCI BDFs from the node inventory) and
  an allocation policy (``first-fit`` like a plain kubelet, or ``topology`` = GetPreferredAllocation
  backed by :mod:`gpumounter_amd.hw.topology`);
* the kubelet's PodResources ledger (which pod/container holds which device IDs);
* per-container cgroup directories laid out as kubelet+runc would (cgroup v1 ``devices`` or v2
  unified; ``cgroupfs`` or ``systemd`` driver) with ``cgroup.procs`` and — for v1 —
  ``devices.allow/deny/list``;
* a per-container root filesystem directory (stands in for ``/proc/<pid>/root``) with ``/dev``.
"""
from __future__ import annotations

import json
import os
import random
import secrets
import shutil
import threading
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Sequence, Tuple

from gpumounter_amd.hw import topology
from gpumounter_amd.models.device import AmdGpu, LinkMatrix
from gpumounter_amd.node import checkpoint as ckpt
from gpumounter_amd.node.checkpoint import CHECKPOINT_NAME
from gpumounter_amd.models.pod import QOS_BESTEFFORT, QOS_BURSTABLE, qos_class

FAKE_MARKER = ".gm_fake"
# runc's default device allow-list (OCI spec defaults), v1 devices.list syntax
RUNTIME_DEFAULT_RULES = [
    "c *:* m", "b *:* m", "c 1:3 rwm", "c 1:5 rwm", "c 1:7 rwm", "c 1:8 rwm", "c 1:9 rwm",
    "c 5:0 rwm", "c 5:1 rwm", "c 5:2 rwm", "c 136:* rwm", "c 10:200 rwm",
]


@dataclass
class Container:
    pod_ns: str
    pod_name: str
    pod_uid: str
    name: str
    id: str
    runtime: str
    cgroup_dir: str
    root_dir: str
    pids: List[int] = field(default_factory=list)


def _esc(s: str) -> str:
    return s.replace("-", "_")


class FakeNode:
    def __init__(self, name: str, workdir: str, gpus: Sequence[AmdGpu],
                 links: Optional[LinkMatrix] = None, resource: str = "amd.com/gpu",
                 cgroup_mode: str = "v1", cgroup_driver: str = "cgroupfs",
                 runtime: str = "containerd", device_id_kind: str = "bdf",
                 alloc_policy: str = "first-free", labels: Optional[Dict[str, str]] = None,
                 cgroup_root: str = "", kernel_fs_dir: str = "") -> None:
        self.name = name
        self.resource = resource
        self.gpus = list(gpus)
        self.links = links
        self.cgroup_mode = cgroup_mode
        self.cgroup_driver = cgroup_driver
        self.runtime = runtime
        if alloc_policy not in ("first-free", "random", "topology"):
            raise ValueError(f"alloc_policy {alloc_policy!r}: first-free | random | topology")
        self.alloc_policy = alloc_policy
        self._rng = random.Random(f"{name}-devices")
        self.device_id_kind = device_id_kind
        self.labels = {"kubernetes.io/hostname": name, "gpu-mounter-enable": "enable"}
        self.labels.update(labels or {})
        self.workdir = workdir
        # kernel_fs_dir: where the trees a real node keeps in memory live — cgroupfs (kernfs),
        # each container's /dev and the host's /dev (tmpfs/devtmpfs). A tmpfs there (bench.py)
        # gives their emulation memory-speed file operations, as on a real node; the worker's
        # own state (the journal, on disk on a real node) stays under ``workdir``.
        kdir = kernel_fs_dir or workdir
        # cgroup_root given: a REAL cgroup2 mount (privileged tests) — directories are real
        # cgroups, cgroup.procs moves real processes, nothing else is written into it
        self.real_cgroups = bool(cgroup_root)
        self.cgroup_root = cgroup_root or os.path.join(kdir, "cgroup")
        self.rootfs_root = os.path.join(kdir, "rootfs")
        os.makedirs(self.cgroup_root, exist_ok=True)
        os.makedirs(self.rootfs_root, exist_ok=True)
        # the worker's node-local state (injection journal) and the node's own /dev, holding an
        # (emulated) node for every GPU like a real host; containers that bind-mount the host's
        # /dev (hostPath /dev, privileged) see exactly this directory
        self.state_dir = os.path.join(workdir, "state")
        self.host_root = os.path.join(kdir, "hostroot")
        self.host_dev = os.path.join(self.host_root, "dev")
        self._populate_host_dev()
        if self.real_cgroups:
            pass
        elif cgroup_mode == "v2":
            with open(os.path.join(self.cgroup_root, "cgroup.controllers"), "w") as fh:
                fh.write("cpuset cpu io memory pids\n")
        else:
            os.makedirs(os.path.join(self.cgroup_root, "devices"), exist_ok=True)
        self.images: set = set()
        self._lock = threading.RLock()
        # device id → (ns, pod, container), and the owning pod's UID
        self.allocated: Dict[str, Tuple[str, str, str]] = {}
        self.alloc_uid: Dict[str, str] = {}
        # pods deleted at the apiserver whose teardown the kubelet has not run yet: their
        # devices are freed by that teardown or, whichever comes first, by the next Allocate
        # (the device manager's UpdateAllocatedDevices drops pods that are no longer active)
        self.pending_release: set = set()
        # the device manager's checkpoint, rewritten (tmp + rename) after every allocation
        # change like the kubelet's (node/checkpoint.py); write_checkpoint=False models a kubelet
        # that does not maintain it
        self.plugin_dir = os.path.join(workdir, "device-plugins")
        os.makedirs(self.plugin_dir, exist_ok=True)
        self.checkpoint_path = os.path.join(self.plugin_dir, CHECKPOINT_NAME)
        self.write_checkpoint = True
        # lazy_checkpoint models the real device manager more closely: it drops a deleted
        # Pod's devices from its books (and the checkpoint) only at the next Allocate
        # (UpdateAllocatedDevices), so the file keeps listing the Pod until then. What the
        # released devices were last checkpointed as: device → (pod uid, container)
        self.lazy_checkpoint = False
        self._stale: Dict[str, Tuple[str, str]] = {}
        self.containers: Dict[str, Container] = {}  # container id → Container
        self.alloc_log: Deque[Tuple[str, str, List[str]]] = deque(maxlen=4096)
        # a registered device plugin (FakeKubelet device manager) replaces allocate()
        self.plugin = None
        self.unhealthy: set = set()
        # "device-plugin": GPUs are the extended resource the kubelet's device manager hands
        # out; "dra": a DRA driver publishes them in a ResourceSlice (fakes/dra.py) and the
        # device manager never sees them (no checkpoint entries)
        self.gpu_api = "device-plugin"
        # a kubelet's device manager writes its checkpoint when it starts (registered devices,
        # no allocations yet), not only at the first Allocate
        self._checkpoint()

    def _populate_host_dev(self) -> None:
        os.makedirs(os.path.join(self.host_dev, "dri"), exist_ok=True)
        nodes = [("kfd", 0, 0)]
        for g in self.gpus:
            nodes.append((f"dri/renderD{g.render_minor}", 226, g.render_minor))
            nodes.append((f"dri/card{g.card_minor}", 226, g.card_minor))
        for rel, ma, mi in nodes:
            with open(os.path.join(self.host_dev, rel), "w") as fh:
                fh.write(f"gm-chr {ma}:{mi}\n")

    def host_dev_nodes(self) -> List[str]:
        out = []
        for d, _, files in os.walk(self.host_dev):
            out += [os.path.relpath(os.path.join(d, f), self.host_dev) for f in files]
        return sorted(out)

    @staticmethod
    def shares_host_dev(pod: dict, cname: str) -> bool:
        """Privileged containers and containers mounting the hostPath /dev at /dev see the
        host's device directory itself."""
        vols = {v.get("name"): (v.get("hostPath") or {}).get("path")
                for v in pod.get("spec", {}).get("volumes", []) or []}
        for c in pod.get("spec", {}).get("containers", []) or []:
            if c.get("name") != cname:
                continue
            if (c.get("securityContext") or {}).get("privileged") is True:
                return True
            for m in c.get("volumeMounts", []) or []:
                if m.get("mountPath") == "/dev" and vols.get(m.get("name")) == "/dev":
                    return True
        return False

    # ------------------------------------------------------------------------ device plugin
    def device_id(self, g: AmdGpu) -> str:
        return {"bdf": g.bdf, "uuid": g.uuid, "render": f"renderD{g.render_minor}"}[
            self.device_id_kind]

    @property
    def capacity(self) -> int:
        return len(self.gpus)

    def device_ids(self) -> List[str]:
        return [self.device_id(g) for g in self.gpus]

    def free_ids(self) -> List[str]:
        with self._lock:
            self.release_pending()
            return [d for d in self.device_ids() if d not in self.allocated]

    def _checkpoint(self) -> None:
        if not self.write_checkpoint:
            return
        per: Dict[Tuple[str, str], Dict[int, List[str]]] = {}
        entries = [(d, self.alloc_uid.get(d, ""), c)
                   for d, (_, _, c) in sorted(self.allocated.items())]
        entries += [(d, uid, c) for d, (uid, c) in sorted(self._stale.items())
                    if d not in self.allocated]
        for d, uid, c in entries:
            if uid:
                per.setdefault((uid, c), {}).setdefault(max(self.numa_of(d), 0), []).append(d)
        ckpt.write_atomic(self.checkpoint_path, ckpt.render(
            [(uid, c, self.resource, ids) for (uid, c), ids in sorted(per.items())],
            {self.resource: self.device_ids()}))

    def allocate(self, ns: str, pod: str, container: str, n: int,
                 uid: str = "") -> Optional[List[str]]:
        """kubelet device-manager Allocate; returns device IDs or None (insufficient).

        Which devices a pod gets is the device plugin's business, and no plugin shipped for
        ``amd.com/gpu`` reads gpumounter's ``preferred-devices`` annotation (the kubelet never
        passes pod annotations to a plugin), so this fake does not read it either:

        * ``first-free`` (default): free devices in device order;
        * ``random``: the kubelet's own choice when the plugin offers no
          GetPreferredAllocation — it takes devices from a Go set, whose iteration order is
          unspecified (seeded here, so runs repeat);
        * ``topology``: a plugin with its own GetPreferredAllocation (the ROCm plugin's
          best-effort policy): the best-connected free set, with no idea which GPUs the pod
          that will receive them already holds.

        Only gpumounter's own device plugin (``deviceplugin/plugin.py``, registered through
        the FakeKubelet's device manager) steers placeholders to a chosen set."""
        with self._lock:
            self.release_pending()
            if self._stale:                  # UpdateAllocatedDevices: inactive pods dropped
                self._stale.clear()
                self._checkpoint()
            free = [g for g in self.gpus if self.device_id(g) not in self.allocated]
            if len(free) < n:
                return None
            chosen: List[AmdGpu]
            if self.alloc_policy == "topology":
                plc = topology.choose(free, n, self.links, policy="xgmi")
                chosen = [next(g for g in free if g.index == i) for i in plc.chosen]
            elif self.alloc_policy == "random":
                chosen = self._rng.sample(free, n)
            else:
                chosen = free[:n]
            ids = [self.device_id(g) for g in chosen]
            for d in ids:
                self.allocated[d] = (ns, pod, container)
                self.alloc_uid[d] = uid
            self.alloc_log.append((ns, pod, ids))
            self._checkpoint()
            return ids

    def record(self, ns: str, pod: str, container: str, ids: Sequence[str],
               uid: str = "") -> bool:
        """Commit an allocation chosen elsewhere (device-plugin path); False if any is taken."""
        with self._lock:
            self.release_pending()
            if self._stale:
                self._stale.clear()
                self._checkpoint()
            if any(d in self.allocated for d in ids):
                return False
            for d in ids:
                self.allocated[d] = (ns, pod, container)
                self.alloc_uid[d] = uid
            self.alloc_log.append((ns, pod, list(ids)))
            self._checkpoint()
            return True

    def release_pending(self) -> None:
        with self._lock:
            while self.pending_release:
                self.release_pod(*self.pending_release.pop())

    def release_pod(self, ns: str, pod: str, uid: str = "") -> List[str]:
        """Free the pod's devices (``uid``: only that incarnation's — a Pod re-created under
        the same name keeps its own)."""
        with self._lock:
            self.pending_release.discard((ns, pod))
            ids = [d for d, (n, p, _) in self.allocated.items() if n == ns and p == pod
                   and (not uid or self.alloc_uid.get(d, "") == uid)]
            for d in ids:
                if self.lazy_checkpoint and self.alloc_uid.get(d):
                    self._stale[d] = (self.alloc_uid[d], self.allocated[d][2])
                del self.allocated[d]
                self.alloc_uid.pop(d, None)
            if ids and not self.lazy_checkpoint:
                self._checkpoint()
            return ids

    def ledger(self) -> Dict[Tuple[str, str], Dict[str, Dict[str, List[str]]]]:
        """(ns, pod) → container → resource → device IDs (PodResources List view)."""
        out: Dict[Tuple[str, str], Dict[str, Dict[str, List[str]]]] = {}
        with self._lock:
            for d, (ns, pod, c) in sorted(self.allocated.items()):
                out.setdefault((ns, pod), {}).setdefault(c, {}).setdefault(
                    self.resource, []).append(d)
        return out

    def numa_of(self, device_id: str) -> int:
        for g in self.gpus:
            if self.device_id(g) == device_id:
                return g.numa_node
        return -1

    # ------------------------------------------------------------------------ runtime
    def pod_cgroup_rel(self, pod: dict) -> str:
        uid = pod["metadata"]["uid"]
        qos = qos_class(pod)
        if self.cgroup_driver == "systemd":
            parts = ["kubepods.slice"]
            if qos == QOS_BURSTABLE:
                parts.append("kubepods-burstable.slice")
                parts.append(f"kubepods-burstable-pod{_esc(uid)}.slice")
            elif qos == QOS_BESTEFFORT:
                parts.append("kubepods-besteffort.slice")
                parts.append(f"kubepods-besteffort-pod{_esc(uid)}.slice")
            else:
                parts.append(f"kubepods-pod{_esc(uid)}.slice")
            return "/".join(parts)
        parts = ["kubepods"]
        if qos == QOS_BURSTABLE:
            parts.append("burstable")
        elif qos == QOS_BESTEFFORT:
            parts.append("besteffort")
        parts.append(f"pod{uid}")
        return "/".join(parts)

    def container_cgroup_leaf(self, cid: str) -> str:
        if self.cgroup_driver == "systemd":
            prefix = {"docker": "docker", "containerd": "cri-containerd", "cri-o": "crio"}[
                self.runtime]
            return f"{prefix}-{cid}.scope"
        return cid

    def start_container(self, pod: dict, cname: str, pids: Sequence[int] = ()) -> Container:
        cid = secrets.token_hex(32)
        rel = self.pod_cgroup_rel(pod) + "/" + self.container_cgroup_leaf(cid)
        base = os.path.join(self.cgroup_root, "devices") if self.cgroup_mode == "v1" \
            else self.cgroup_root
        cg = os.path.join(base, rel)
        os.makedirs(cg, exist_ok=True)
        if self.real_cgroups:
            for p in pids:   # the kernel takes one PID per write
                with open(os.path.join(cg, "cgroup.procs"), "w") as fh:
                    fh.write(str(p))
        else:
            with open(os.path.join(cg, FAKE_MARKER), "w") as fh:
                fh.write(json.dumps({"mode": self.cgroup_mode, "container": cid}))
            with open(os.path.join(cg, "cgroup.procs"), "w") as fh:
                fh.write("".join(f"{p}\n" for p in pids))
        if self.cgroup_mode == "v1" and not self.real_cgroups:
            for f in ("devices.allow", "devices.deny"):
                open(os.path.join(cg, f), "w").close()
            with open(os.path.join(cg, "devices.list"), "w") as fh:
                fh.write("\n".join(RUNTIME_DEFAULT_RULES) + "\n")
        root = os.path.join(self.rootfs_root, cid)
        if self.shares_host_dev(pod, cname):
            os.symlink(self.host_root, root)     # its root's dev/ IS the host's /dev
        else:
            os.makedirs(os.path.join(root, "dev"), exist_ok=True)
        c = Container(pod["metadata"]["namespace"], pod["metadata"]["name"],
                      pod["metadata"]["uid"], cname, cid, self.runtime, cg, root, list(pids))
        with self._lock:
            self.containers[cid] = c
        return c

    def set_container_pids(self, cid: str, pids: Sequence[int]) -> None:
        with self._lock:
            c = self.containers[cid]
            c.pids = list(pids)
            with open(os.path.join(c.cgroup_dir, "cgroup.procs"), "w") as fh:
                fh.write("".join(f"{p}\n" for p in pids))

    def stop_container(self, cid: str) -> None:
        """One container exits: its cgroup and root filesystem go (a restart starts a fresh
        container with a new id, as a runtime does)."""
        with self._lock:
            c = self.containers.pop(cid, None)
        if c is None:
            return
        shutil.rmtree(c.cgroup_dir, ignore_errors=True)
        if os.path.islink(c.root_dir):
            os.unlink(c.root_dir)
        else:
            shutil.rmtree(c.root_dir, ignore_errors=True)

    def stop_pod_containers(self, ns: str, pod: str, uid: str = "") -> None:
        with self._lock:
            for cid, c in list(self.containers.items()):
                if c.pod_ns == ns and c.pod_name == pod and (not uid or c.pod_uid == uid):
                    shutil.rmtree(c.cgroup_dir, ignore_errors=True)
                    # prune empty pod-level cgroup dir like kubelet does
                    parent = os.path.dirname(c.cgroup_dir)
                    try:
                        if not [e for e in os.listdir(parent) if not e.startswith(".")]:
                            shutil.rmtree(parent, ignore_errors=True)
                    except OSError:
                        pass
                    if os.path.islink(c.root_dir):
                        os.unlink(c.root_dir)
                    else:
                        shutil.rmtree(c.root_dir, ignore_errors=True)
                    del self.containers[cid]

    def container(self, cid: str) -> Optional[Container]:
        with self._lock:
            return self.containers.get(cid)

    # ------------------------------------------------------------------------ audit helpers
    @staticmethod
    def v1_effective_extra_rules(cgdir: str) -> Dict[str, int]:
        """Net allow count per rule written by the worker (allow lines minus deny lines)."""
        net: Dict[str, int] = {}
        for fname, sign in (("devices.allow", 1), ("devices.deny", -1)):
            try:
                with open(os.path.join(cgdir, fname)) as fh:
                    for line in fh:
                        line = line.strip()
                        if line:
                            net[line] = net.get(line, 0) + sign
            except FileNotFoundError:
                pass
        return net

    def container_devices(self, cid: str) -> List[str]:
        """Device node paths present in a container's /dev (relative, sorted)."""
        c = self.container(cid)
        if c is None:
            return []
        out = []
        dev = os.path.join(c.root_dir, "dev")
        for dirpath, _, files in os.walk(dev):
            for f in files:
                out.append(os.path.relpath(os.path.join(dirpath, f), c.root_dir))
        return sorted(out)
