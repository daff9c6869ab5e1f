"""Reference-protocol emulation — the *reference's* call sequence on the same hermetic cluster.

The reference cannot run here (Go, NVIDIA, a real cluster: SURVEY §0.1), and it publishes no
numbers. To still have an apples-to-apples comparison, this module re-enacts its
control flow step for step, mapped to AMD devices, on the same fake apiserver/kubelet/cgroupfs:

master (reference: cmd/GPUMounter-master/main.go)
  * per request: ``Pods.Get`` + ``Pods.List(kube-system, app=gpu-mounter-worker)`` (52, 255)
  * a new insecure gRPC connection per request, closed afterwards (82-96, 185-199)
worker (reference: pkg/server/gpu-mount/server.go, pkg/util/gpu/allocator/allocator.go)
  * ``Pods.Get`` of the target, mount type via a fresh kubelet dial + ``List`` (collector.go:98)
  * slave pods created *sequentially*, image ``alpine:latest`` (pull policy Always), a ``sh``
    sleep loop that ignores SIGTERM, cross-namespace ownerReference (allocator.go:49-60,189-234)
  * readiness by a tight ``Pods.Get`` loop over all slaves until Running (236-282)
  * one fresh kubelet dial + ``List`` per slave pod to read its device IDs (86-94)
  * per GPU: ``fork sh -c "echo 'c MAJ:MIN rw' > devices.allow"`` and
    ``fork nsenter … sh -c "mknod …"`` (util.go:37-67) — here two nested shells because the
    benchmark host is unprivileged (no nsenter/mknod); the marker file stands in for the node
  * removal: two kubelet dials, busy check, ``devices.deny`` + ``rm`` forks, then
    ``Pods.Delete`` with *default* options (30 s grace; the sh loop ignores SIGTERM) and a tight
    ``Pods.Get`` loop until NotFound (128-156, 284-317)
Everything is labelled *emulated* wherever it is reported.
"""
from __future__ import annotations

import asyncio
import os
import secrets
from typing import List

import grpc

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.api.podresources import V1ALPHA1
from gpumounter_amd.cluster.kube import NotFound
from gpumounter_amd.master.app import ANN_WORKER_PORT, Master
from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.device import AmdGpu, gpus_by_key, normalize_device_id
from gpumounter_amd.models.pod import running_containers
from gpumounter_amd.utils import trace


class RefMaster(Master):
    """Master with the reference's per-request worker discovery and dialing."""

    async def _locate(self, ns, name, fresh=False):
        try:
            pod = await self.kube.get_pod(ns, name)
        except NotFound:
            return None, None, (404, f"No pod: {name} in namespace: {ns}", {}), False
        items, _ = await self.kube.list_pods(self.cfg.worker_namespace, self.cfg.worker_label)
        node = podu.node_of(pod)
        for w in items:
            if podu.node_of(w) == node:
                port = (w["metadata"].get("annotations") or {}).get(ANN_WORKER_PORT, "1200")
                return pod, f"{w['status']['podIP']}:{port}", None, False
        return pod, None, (500, "Service Internal Error", {}), False

    class _OneShot:
        def __init__(self, target):
            self.ch = grpc.aio.insecure_channel(target)

        def unary_unary(self, path, request_serializer, response_deserializer):
            inner = self.ch.unary_unary(path, request_serializer=request_serializer,
                                        response_deserializer=response_deserializer)
            ch = self.ch

            async def call(req, timeout=None):
                try:
                    return await inner(req)            # reference: context.TODO(), no deadline
                finally:
                    await ch.close()
            return call

    def __init__(self, cfg, kube=None):
        super().__init__(cfg, kube)
        self.workers.channel = lambda target: RefMaster._OneShot(target)


async def _sh(cmd: str) -> None:
    p = await asyncio.create_subprocess_exec("sh", "-c", cmd, stdout=asyncio.subprocess.DEVNULL,
                                             stderr=asyncio.subprocess.PIPE)
    _, err = await p.communicate()
    if p.returncode != 0:
        raise RuntimeError(f"`{cmd}` failed: {err.decode().strip()}")


class RefProtocolService:
    """Drop-in replacement for GpuMountService.add_gpu/remove_gpu with the reference's flow."""

    def __init__(self, svc) -> None:
        self.svc = svc
        self.cfg = svc.cfg
        self.kube = svc.kube
        self.inv = svc.inv

    # ------------------------------------------------------------------ kubelet: dial per query
    async def _ledger(self):
        ch = grpc.aio.insecure_channel(f"unix://{self.cfg.kubelet_socket}")
        try:
            stub = ch.unary_unary(V1ALPHA1.LIST,
                                  request_serializer=V1ALPHA1.ListPodResourcesRequest.SerializeToString,
                                  response_deserializer=V1ALPHA1.ListPodResourcesResponse.FromString)
            resp = await stub(V1ALPHA1.ListPodResourcesRequest(), timeout=10)
        finally:
            await ch.close()
        out = {}
        for pr in resp.pod_resources:
            for c in pr.containers:
                for d in c.devices:
                    if d.resource_name == self.cfg.resource_name:
                        out.setdefault((pr.namespace, pr.name), []).extend(d.device_ids)
        return out

    async def _pod_gpus(self, name: str, ns: str):
        """GetPodGPUResources: the pod's GPUs + (substring-matched) slave GPUs."""
        led = await self._ledger()
        keys = gpus_by_key(self.inv.gpus())
        out = []
        for (pns, pname), ids in led.items():
            mine = (pname == name and pns == ns) or (
                name + "-slave-pod-" in pname and pns == self.cfg.pool_namespace)
            if mine:
                for d in ids:
                    g = keys[normalize_device_id(d)]
                    g.pod_name, g.namespace = pname, pns
                    out.append(g)
        return out

    async def _mount_type(self, pod) -> str:
        gs = await self._pod_gpus(podu.name_of(pod), podu.ns_of(pod))
        if not gs:
            return "no-mount"
        slaves = {g.pod_name for g in gs if g.pod_name != podu.name_of(pod)}
        return "entire-mount" if len(slaves) < len(gs) else "single-mount"

    # ------------------------------------------------------------------ slave pods
    def _slave(self, owner, n):
        name = f"{podu.name_of(owner)}-slave-pod-{secrets.token_hex(3)}"
        return {"metadata": {"name": name, "namespace": self.cfg.pool_namespace,
                             "labels": {"app": "gpu-pool"},
                             "ownerReferences": [{"apiVersion": "v1", "kind": "Pod",
                                                  "name": podu.name_of(owner),
                                                  "uid": podu.uid_of(owner),
                                                  "blockOwnerDeletion": True,
                                                  "controller": True}]},
                "spec": {"containers": [{
                    "name": "gpu-container", "image": "alpine:latest", "command": ["/bin/sh"],
                    "args": ["-c", "while true; do echo this is a gpu pool container; "
                                   "sleep 10;done"],
                    "resources": {"limits": {self.cfg.resource_name: str(n)}}}],
                    "nodeSelector": {"kubernetes.io/hostname": podu.node_of(owner)}}}

    async def _check_create(self, names: List[str]) -> str:
        while True:  # tight loop, no sleep (allocator.go:246-281); yield to the event loop only
            done = True
            for n in names:
                try:
                    p = await self.kube.get_pod(self.cfg.pool_namespace, n)
                except NotFound:
                    continue
                if podu.phase_of(p) == "Running":
                    continue
                conds = p["status"].get("conditions") or []
                if conds and conds[0].get("reason") == "Unschedulable":
                    return "InsufficientGPU"
                done = False
            if done:
                return "SuccessfullyCreated"
            await asyncio.sleep(0)

    async def _check_delete(self, names: List[str]) -> None:
        while True:
            alive = False
            for n in names:
                try:
                    await self.kube.get_pod(self.cfg.pool_namespace, n)
                    alive = True
                except NotFound:
                    pass
            if not alive:
                return
            await asyncio.sleep(0)

    # ------------------------------------------------------------------ node ops via shells
    def _paths(self, pod):
        c = running_containers(pod)[0]                      # ContainerStatuses[0] only
        cg = self.svc.hm.resolver.container_dir(pod, c)
        root = os.path.join(self.cfg.container_root_prefix, c.id)
        return cg, root

    async def _mount(self, pod, g: AmdGpu, first: bool) -> None:
        cg, root = self._paths(pod)
        nodes = g.device_nodes(self.cfg.drm_major, False)
        if first:
            nodes = [self.svc.hm.kfd()] + nodes
        for n in nodes:
            await _sh(f"echo 'c {n.major}:{n.minor} rw' >> {cg}/devices.allow")
            path = root + n.path
            await _sh("sh -c " + repr(f"mkdir -p {os.path.dirname(path)} && "
                                      f"printf 'gm-chr {n.major}:{n.minor}\\n' > {path} && "
                                      f"chmod 666 {path}"))

    async def _unmount(self, pod, g: AmdGpu, last: bool) -> None:
        cg, root = self._paths(pod)
        nodes = g.device_nodes(self.cfg.drm_major, False)
        if last:
            nodes = nodes + [self.svc.hm.kfd()]
        for n in nodes:
            await _sh(f"echo 'c {n.major}:{n.minor} rw' >> {cg}/devices.deny")
            await _sh("sh -c " + repr(f"rm {root + n.path}"))

    # ------------------------------------------------------------------ RPCs
    async def add_gpu(self, req):
        with trace.span("attach") as root:
            try:
                pod = await self.kube.get_pod(req.namespace, req.pod_name)
            except NotFound:
                return api.AddGPUResponse(add_gpu_result=api.ADD_POD_NOT_FOUND)
            mt = await self._mount_type(pod)
            if mt == "entire-mount" or (mt != "no-mount" and req.is_entire_mount):
                raise RuntimeError("FailedCreated")
            n = req.gpu_num
            per = n if req.is_entire_mount else 1
            names = []
            for _ in range(n // per):                        # sequential creates
                body = self._slave(pod, per)
                created = await self.kube.create_pod(self.cfg.pool_namespace, body)
                names.append(created["metadata"]["name"])
            res = await self._check_create(names)
            if res != "SuccessfullyCreated":
                for nm in names:
                    await self.kube.delete_pod(self.cfg.pool_namespace, nm, grace_period_s=0)
                return api.AddGPUResponse(add_gpu_result=api.ADD_INSUFFICIENT)
            gpus = []
            for nm in names:                                  # kubelet dial per slave
                gpus += await self._pod_gpus(nm, self.cfg.pool_namespace)
            had = await self._pod_gpus(podu.name_of(pod), podu.ns_of(pod))
            first = len(had) == len(gpus)
            for i, g in enumerate(gpus):
                await self._mount(pod, g, first and i == 0)
        resp = api.AddGPUResponse(add_gpu_result=api.ADD_SUCCESS, total_ms=root.duration_ms)
        for g in gpus:
            resp.devices.add(uuid=g.uuid, bdf=g.bdf, index=g.index,
                             render_minor=g.render_minor, numa_node=g.numa_node)
        return resp

    async def remove_gpu(self, req):
        with trace.span("detach") as root:
            try:
                pod = await self.kube.get_pod(req.namespace, req.pod_name)
            except NotFound:
                return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_POD_NOT_FOUND)
            gs = await self._pod_gpus(podu.name_of(pod), podu.ns_of(pod))
            mt = await self._mount_type(pod)
            want = {normalize_device_id(u) for u in req.uuids}
            sel = [g for g in gs if (mt == "entire-mount" or want & set(g.ledger_keys()))
                   and g.pod_name != podu.name_of(pod)]
            if len(sel) != len(req.uuids):
                return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_GPU_NOT_FOUND)
            hot_left = len([g for g in gs if g.pod_name != podu.name_of(pod)]) - len(sel)
            for i, g in enumerate(sel):
                await self._unmount(pod, g, last=hot_left == 0 and i == len(sel) - 1)
            names = sorted({g.pod_name for g in sel})
            for nm in names:                                  # default DeleteOptions
                await self.kube.delete_pod(self.cfg.pool_namespace, nm)
            await self._check_delete(names)
        return api.RemoveGPUResponse(remove_gpu_result=api.REMOVE_SUCCESS,
                                     total_ms=root.duration_ms)


def install(lc) -> None:
    """Switch a running LocalCluster to the reference protocol (master + every worker)."""
    for h in lc.nodes.values():
        ref = RefProtocolService(h.worker.service)
        h.worker.service.add_gpu = ref.add_gpu
        h.worker.service.remove_gpu = ref.remove_gpu
    lc.master.workers.channel = lambda target: RefMaster._OneShot(target)
    lc.master._locate = RefMaster._locate.__get__(lc.master)


# ------------------------------------------------------------------------------ as daemons
async def _serve(role: str, cfg) -> None:
    """The reference protocol in a worker or master *process* (ProcessCluster, protocol=
    "reference"): the production daemon with the same substitutions :func:`install` makes."""
    import signal

    from gpumounter_amd.worker.server import Worker

    if role == "worker":
        d = Worker(cfg)
        ref = RefProtocolService(d.service)
        d.service.add_gpu = ref.add_gpu
        d.service.remove_gpu = ref.remove_gpu
    else:
        d = Master(cfg)
        d.workers.channel = lambda target: RefMaster._OneShot(target)
        d._locate = RefMaster._locate.__get__(d)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    await d.start()
    try:
        await stop.wait()
    finally:
        await d.stop()


def main(argv=None) -> int:
    """``python -m gpumounter_amd.fakes.refproto worker|master`` (GM_* env as the daemons)."""
    import sys

    from gpumounter_amd.utils import log
    from gpumounter_amd.utils.config import Config

    role = (argv or sys.argv[1:])[0]
    cfg = Config.load()
    log.setup(cfg.log_level, cfg.log_json, cfg.log_file)
    asyncio.run(_serve(role, cfg))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
