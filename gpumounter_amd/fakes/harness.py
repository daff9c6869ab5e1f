"""LocalCluster: a complete hermetic deployment in one asyncio loop.

fake apiserver (HTTP) + per-node fake kubelet (PodResources gRPC on a unix socket) + per-node
:class:`~gpumounter_amd.worker.server.Worker` (real gRPC server, real C++ host ops against a
temp-dir cgroupfs/rootfs) + :class:`~gpumounter_amd.master.app.Master` (real HTTP server).
Only the Kubernetes control plane is simulated; every byte between master, worker, kubelet and
apiserver crosses a real socket, and the node operations run the production code paths.

The GPU inventory comes from the amdsmi shim: the bundled mock on CPU hosts, the real
``libamd_smi`` on an MI355X box (``amdsmi_lib=""``).
"""
from __future__ import annotations

import asyncio
import os
import shutil
import tempfile
import threading
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import aiohttp
import yaml
from aiohttp import web

from gpumounter_amd.fakes.apiserver import FakeCluster, LatencyModel
from gpumounter_amd.fakes.kubelet import FakeKubelet
from gpumounter_amd.fakes.node import FakeNode
from gpumounter_amd.hw.inventory import Inventory
from gpumounter_amd.master.app import ANN_WIRE_PORT, ANN_WORKER_PORT, Master
from gpumounter_amd.utils.config import Config
from gpumounter_amd.worker.server import Worker


_DEPLOY_PRIORITY = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "deploy", "placeholder-priority.yaml")


def deploy_priority_classes() -> List[dict]:
    """The PriorityClass objects of the shipped deploy."""
    with open(_DEPLOY_PRIORITY, encoding="utf-8") as fh:
        return [d for d in yaml.safe_load_all(fh) if d]


@dataclass
class NodeHandle:
    name: str
    node: FakeNode
    kubelet: FakeKubelet
    worker: Optional[Worker] = None
    cfg: Optional[Config] = None


class LocalCluster:
    def __init__(self, n_nodes: int = 1, amdsmi_lib: str = "mock", cgroup_mode: str = "v1",
                 cgroup_driver: str = "cgroupfs", runtime: str = "containerd",
                 latency: Optional[LatencyModel] = None, gc_mode: str = "modern",
                 workdir: str = "", placeholder_namespace_mode: str = "pool",
                 alloc_policy: str = "first-free", device_id_kind: str = "bdf",
                 devnode_mode: str = "emulate", reconcile_period_s: float = 0.0,
                 start_master: bool = True, worker_overrides: Optional[dict] = None,
                 node_gpu_bdfs: Optional[List[str]] = None,
                 master_overrides: Optional[dict] = None,
                 device_plugin: bool = False, cgroup_root: str = "",
                 kfd_major: int = 0, start_workers: bool = True,
                 kubelet_rate_limit: Optional[tuple] = (100.0, 10),
                 kubelet_limit_mode: str = "enforce", gpu_api: str = "device-plugin",
                 app_hook: Optional[Callable[[web.Application], None]] = None,
                 kernel_fs_dir: str = "", priority_classes: bool = True,
                 lazy_checkpoint: bool = False) -> None:
        self.n_nodes = n_nodes
        # the device manager keeps a deleted Pod in its checkpoint until the next Allocate, as
        # a real kubelet does (fakes/node.py FakeNode.lazy_checkpoint)
        self.lazy_checkpoint = lazy_checkpoint
        # apply the shipped deploy's PriorityClasses (deploy/placeholder-priority.yaml), as
        # `kubectl apply -k deploy/` does; False: a cluster where they were never applied
        self.priority_classes = priority_classes
        self.kernel_fs_dir = kernel_fs_dir     # see FakeNode; removed by stop()
        self.amdsmi_lib = amdsmi_lib
        self.cgroup_mode = cgroup_mode
        self.cgroup_driver = cgroup_driver
        self.runtime = runtime
        self.cluster = FakeCluster(latency, gc_mode)
        self._own_workdir = not workdir
        self.workdir = workdir or tempfile.mkdtemp(prefix="gm-cluster-")
        self.placeholder_namespace_mode = placeholder_namespace_mode
        self.alloc_policy = alloc_policy
        self.device_id_kind = device_id_kind
        self.devnode_mode = devnode_mode
        self.reconcile_period_s = reconcile_period_s
        self.start_master = start_master
        self.start_workers = start_workers
        self.app_hook = app_hook
        self.worker_overrides = worker_overrides or {}
        self.master_overrides = master_overrides or {}
        self.device_plugin = device_plugin
        self.real_cgroup_root = cgroup_root   # privileged tests: a real cgroup2 mount
        self.kfd_major = kfd_major
        self.kubelet_rate_limit = kubelet_rate_limit
        self.kubelet_limit_mode = kubelet_limit_mode
        self.gpu_api = gpu_api      # "dra": GPUs published by a DRA driver (fakes/dra.py)
        self.node_gpu_bdfs = [b.lower() for b in node_gpu_bdfs] if node_gpu_bdfs else None
        self.nodes: Dict[str, NodeHandle] = {}
        self.master: Optional[Master] = None
        self.api_runner: Optional[web.AppRunner] = None
        self.api_url = ""
        self.master_url = ""
        self.inventory: Optional[Inventory] = None
        self.session: Optional[aiohttp.ClientSession] = None

    # ------------------------------------------------------------------------ lifecycle
    async def start(self) -> "LocalCluster":
        self.inventory = Inventory(self.amdsmi_lib, self.kfd_major)
        app = self.cluster.app()
        if self.app_hook is not None:
            self.app_hook(app)
        self.api_runner = web.AppRunner(app, access_log=None)
        await self.api_runner.setup()
        site = web.TCPSite(self.api_runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
        self.api_url = f"http://127.0.0.1:{port}"
        self.cluster.loop = asyncio.get_running_loop()
        if self.priority_classes:
            self.cluster.apply_priority_classes(deploy_priority_classes())
        for i in range(self.n_nodes):
            await self._add_node(f"node-{i}")
        if self.start_master:
            mcfg = Config.load(env={}, kube_api=self.api_url, master_host="127.0.0.1",
                               log_json=False,
                               **{"gc_tune": False, "authz_mode": "none",
                                  **self.master_overrides})
            self.master = Master(mcfg)
            await self.master.start(port=0)
            self.master_url = f"http://127.0.0.1:{self.master.port}"
            await self.master.workers.informer.wait_for(
                lambda: all(self.master.workers.target(n) for n in self.nodes), 10)
        self.session = aiohttp.ClientSession()
        return self

    async def _add_node(self, name: str) -> NodeHandle:
        ndir = os.path.join(self.workdir, name)
        os.makedirs(ndir, exist_ok=True)
        gpus = self.inventory.gpus()
        if self.node_gpu_bdfs is not None:
            gpus = [g for g in gpus if g.bdf in self.node_gpu_bdfs]
        node = FakeNode(name, ndir, gpus, self.inventory.links(),
                        cgroup_mode=self.cgroup_mode, cgroup_driver=self.cgroup_driver,
                        runtime=self.runtime, device_id_kind=self.device_id_kind,
                        alloc_policy=self.alloc_policy,
                        cgroup_root=os.path.join(self.real_cgroup_root, name)
                        if self.real_cgroup_root else "",
                        kernel_fs_dir=os.path.join(self.kernel_fs_dir, name)
                        if self.kernel_fs_dir else "")
        node.lazy_checkpoint = self.lazy_checkpoint
        if self.gpu_api == "dra":
            node.gpu_api = "dra"
            node.write_checkpoint = False    # the device manager does not see DRA devices
        self.cluster.add_node(node)
        sock = os.path.join(ndir, "pod-resources", "kubelet.sock")
        kubelet = FakeKubelet(node, sock, plugin_dir=os.path.join(ndir, "device-plugins")
                              if self.device_plugin else "", rate_limit=self.kubelet_rate_limit,
                              limit_mode=self.kubelet_limit_mode)
        await kubelet.start()
        h = NodeHandle(name, node, kubelet)
        self.nodes[name] = h
        if self.start_workers:
            await self.start_worker(name)
        return h

    async def start_worker(self, name: str) -> Worker:
        h = self.nodes[name]
        ov = dict(self.worker_overrides)
        ov.setdefault("gc_tune", False)   # many clusters per test process: freezing would leak
        ov.setdefault("worker_insecure", not ov.get("tls_ca"))   # hermetic: loopback only
        ov.setdefault("state_dir", h.node.state_dir)
        ov.setdefault("host_dev_path", h.node.host_dev)
        # like the periodic sweep, the device guard is opt-in for in-process tests (tests that
        # tamper with a cgroup and then check what the sweep finds would race it)
        ov.setdefault("device_guard_period_s", 0.0)
        if self.device_plugin:
            ov.setdefault("device_plugin", True)
            ov.setdefault("device_plugin_dir", h.kubelet.plugin_dir)
        ov.setdefault("kubelet_checkpoint", h.node.checkpoint_path)
        if self.gpu_api == "dra":
            ov.setdefault("gpu_allocation", "dra")
        cfg = Config.load(env={}, kube_api=self.api_url, node_name=name,
                          kubelet_socket=h.kubelet.socket_path,
                          cgroup_root=h.node.cgroup_root, cgroup_mode=self.cgroup_mode,
                          devnode_mode=self.devnode_mode,
                          container_root_prefix=h.node.rootfs_root
                          if self.devnode_mode == "emulate" else "",
                          amdsmi_lib=self.amdsmi_lib,
                          worker_host="127.0.0.1", worker_port=1, metrics_port=0,
                          placeholder_namespace_mode=self.placeholder_namespace_mode,
                          reconcile_period_s=self.reconcile_period_s, log_json=False,
                          metrics_period_s=ov.pop("metrics_period_s", 0), **ov)
        w = Worker(cfg, inventory=self.inventory)
        await w.start(grpc_port=0, http_port=0, reconcile=self.reconcile_period_s > 0,
                      wire_port=0)
        h.worker, h.cfg = w, cfg
        self.register_worker(name, w.grpc_port, wire_port=w.wire_port)
        return w

    def register_worker(self, name: str, port: int, ip: str = "127.0.0.1",
                        wire_port: int = 0) -> None:
        """Create the worker DaemonSet pod of node ``name`` so the master can discover it
        (``wire_port`` > 0: it also serves gm-wire there, as the DaemonSet annotates)."""
        wp = self.cluster.get("kube-system", f"gpu-mounter-worker-{name}")
        if wp is not None:
            self.cluster._remove("kube-system", wp["metadata"]["name"])  # noqa: SLF001
        # reachable from its first Running version on: a master that read a placeholder
        # address would send its next request to an unroutable IP and wait out the TCP
        # connect (chaos: a 20 s ledger-read stall right after a worker restart)
        self.cluster.create_running_pod("kube-system", {
            "metadata": {"name": f"gpu-mounter-worker-{name}",
                         "labels": {"app": "gpu-mounter-worker"},
                         "annotations": {ANN_WORKER_PORT: str(port),
                                         **({ANN_WIRE_PORT: str(wire_port)}
                                            if wire_port > 0 else {})}},
            "spec": {"containers": [{"name": "worker", "image": "gpumounter-amd:dev"}]}}, name,
            pod_ip=ip)

    async def stop_worker(self, name: str) -> None:
        h = self.nodes[name]
        if h.worker is not None:
            await h.worker.stop()
            h.worker = None

    async def stop(self) -> None:
        if self.session is not None:
            await self.session.close()
        if self.master is not None:
            await self.master.stop()
        for h in self.nodes.values():
            if h.worker is not None:
                await h.worker.stop()
            await h.kubelet.stop()
        for t in list(self.cluster._tasks):  # noqa: SLF001
            t.cancel()
        if self.api_runner is not None:
            await self.api_runner.cleanup()
        if self._own_workdir:
            shutil.rmtree(self.workdir, ignore_errors=True)
        if self.kernel_fs_dir:
            shutil.rmtree(self.kernel_fs_dir, ignore_errors=True)

    async def __aenter__(self) -> "LocalCluster":
        return await self.start()

    async def __aexit__(self, *exc) -> None:
        await self.stop()

    # ------------------------------------------------------------------------ helpers
    def tenant(self, name: str, ns: str = "default", node: str = "node-0",
               containers: Optional[List[str]] = None, gpus: int = 0,
               pids: Optional[Dict[str, List[int]]] = None, qos: str = "besteffort") -> dict:
        cs = []
        for cname in containers or ["main"]:
            c: dict = {"name": cname, "image": "rocm/pytorch:latest",
                       "command": ["sleep", "infinity"]}
            res: dict = {}
            if qos == "guaranteed":
                res = {"limits": {"cpu": "1", "memory": "1Gi"},
                       "requests": {"cpu": "1", "memory": "1Gi"}}
            elif qos == "burstable":
                res = {"requests": {"cpu": "100m"}}
            if gpus:
                res.setdefault("limits", {})["amd.com/gpu"] = str(gpus)
            if res:
                c["resources"] = res
            cs.append(c)
        return self.cluster.create_running_pod(
            ns, {"metadata": {"name": name}, "spec": {"containers": cs}}, node, pids)

    def container_ids(self, ns: str, name: str) -> List[str]:
        pod = self.cluster.get(ns, name)
        return [cs["containerID"].split("://", 1)[1]
                for cs in pod["status"].get("containerStatuses", []) if cs.get("containerID")]

    async def add(self, ns: str, pod: str, n: int, entire: bool = False,
                  accept_json: bool = True, token: str = ""):
        url = (f"{self.master_url}/addgpu/namespace/{ns}/pod/{pod}/gpu/{n}/isEntireMount/"
               f"{'true' if entire else 'false'}")
        headers = {"Accept": "application/json"} if accept_json else {}
        if token:
            headers["Authorization"] = f"Bearer {token}"
        async with self.session.get(url, headers=headers) as r:
            return r.status, (await r.json() if accept_json else await r.text())

    async def remove(self, ns: str, pod: str, uuids: List[str], force: bool = False,
                     accept_json: bool = True, token: str = ""):
        url = (f"{self.master_url}/removegpu/namespace/{ns}/pod/{pod}/force/"
               f"{'true' if force else 'false'}")
        headers = {"Accept": "application/json"} if accept_json else {}
        if token:
            headers["Authorization"] = f"Bearer {token}"
        data = aiohttp.FormData()
        for u in uuids:
            data.add_field("uuids", u)
        async with self.session.post(url, data=data, headers=headers) as r:
            return r.status, (await r.json() if accept_json else await r.text())

    def audit(self, ns: str, pod: str, node: str = "node-0") -> list:
        """Ledger-vs-host consistency issues for one pod (empty list = consistent)."""
        h = self.nodes[node]
        svc = h.worker.service
        p = self.cluster.get(ns, pod)

        async def run():
            st = await svc.pod_state(p)
            return svc.hm.audit(p, st.hot, st.own)
        return run()


class ThreadedCluster:
    """Runs a LocalCluster on a private event loop thread (for sync callers: bench, smoke)."""

    def __init__(self, **kw) -> None:
        self.kw = kw
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self.loop.run_forever, daemon=True,
                                       name="gm-localcluster")
        self.lc: Optional[LocalCluster] = None

    def start(self) -> LocalCluster:
        self.thread.start()
        self.lc = self.call(LocalCluster(**self.kw).start())
        return self.lc

    def call(self, coro, timeout: float = 600):
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    def stop(self) -> None:
        if self.lc is not None:
            self.call(self.lc.stop())
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(timeout=10)
