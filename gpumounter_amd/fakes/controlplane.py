"""The hermetic Kubernetes control plane as a process of its own.

``python -m gpumounter_amd.fakes.controlplane --workdir D --nodes 2 --info D/info.json`` serves the
fake apiserver (with its scheduler and per-node kubelet admission), one fake kubelet PodResources
socket per node and the per-node cgroupfs/rootfs trees — everything a real node agent talks to —
and no gpumounter component. The real daemons (``python -m gpumounter_amd worker|master``) then run
as separate processes against it, configured only through ``GM_*`` environment variables, as in
the DaemonSet/Deployment (see :mod:`gpumounter_amd.fakes.deployment`).

Besides the Kubernetes API it serves these test hooks:
  ``POST /_fake/tenant``  {"name", "ns", "node", "gpus", "containers", "pids"} → a Running pod
  ``POST /_fake/worker``  {"node", "port", "wire_port"}  → the worker DaemonSet pod the master
  discovers
  ``GET  /_fake/kubelet``  → each node's PodResources call counters (served, rejected, over_limit)
  ``POST /_fake/kubelet/restart`` {"node", "down_s"} → kubelet down for down_s, PodResources
                          socket recreated
  ``POST /_fake/recreate`` {"ns", "pod", "gap_s"} → the Pod is deleted and created again under
                          the same name (new UID)
  ``POST /_fake/restart`` {"ns", "pod", "container"} → the container restarts (new id, cgroup, /dev)
  ``POST /_fake/faults``  {"rate", "seed"} → Pod/ResourceClaim requests fail at random (500/503/
                          429, half after taking effect); answers how many were served so far
  ``GET  /_fake/preemptions`` → how many Pods the scheduler preempted, by kind (standby,
                          placeholder booking a tenant's GPU, other)
  ``POST /_fake/user``    {"token", "user", "verbs", "resource", "namespaces"} → a bearer token
                          TokenReview accepts, and an RBAC rule SubjectAccessReview honours
The info file lists the apiserver URL and each node's kubelet socket, cgroup root and rootfs root.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import sys

from aiohttp import web

from gpumounter_amd.fakes.apiserver import LatencyModel
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.utils import log, runtime


def _hooks(lc_ref: list):
    def install(app: web.Application) -> None:
        async def tenant(req: web.Request) -> web.Response:
            b = await req.json()
            pod = lc_ref[0].tenant(b["name"], ns=b.get("ns", "default"),
                                   node=b.get("node", "node-0"), gpus=int(b.get("gpus", 0)),
                                   containers=b.get("containers"), pids=b.get("pids"))
            return web.json_response(pod, status=201)

        async def worker(req: web.Request) -> web.Response:
            b = await req.json()
            lc_ref[0].register_worker(b["node"], int(b["port"]), b.get("ip", "127.0.0.1"),
                                      int(b.get("wire_port", 0)))
            return web.json_response({"ok": True}, status=201)

        async def kubelet(req: web.Request) -> web.Response:
            return web.json_response({n: dict(h.kubelet.calls)
                                      for n, h in lc_ref[0].nodes.items()})

        async def user(req: web.Request) -> web.Response:
            b = await req.json()
            api = lc_ref[0].cluster
            api.add_user(b["token"], b["user"])
            api.grant(b["user"], b.get("verbs", ["create", "delete", "get"]),
                      b.get("resource", "pods/gpumount"), b.get("namespaces", ["*"]))
            return web.json_response({"ok": True}, status=201)

        async def faults(req: web.Request) -> web.Response:
            b = await req.json()
            api = lc_ref[0].cluster
            api.random_failures(float(b.get("rate", 0)), int(b.get("seed", 0)))
            return web.json_response({"served": api.random_faults_served}, status=201)

        async def restart(req: web.Request) -> web.Response:
            b = await req.json()
            cid = lc_ref[0].cluster.restart_container(b.get("ns", "default"), b["pod"],
                                                      b.get("container", "main"))
            return web.json_response({"container_id": cid}, status=201)

        async def kubelet_restart(req: web.Request) -> web.Response:
            from gpumounter_amd.fakes.kubelet import FakeKubelet
            b = await req.json()
            h = lc_ref[0].nodes[b.get("node", "node-0")]
            await h.kubelet.stop()
            await asyncio.sleep(float(b.get("down_s", 0.0)))
            h.kubelet = FakeKubelet(h.node, h.kubelet.socket_path)
            await h.kubelet.start()
            return web.json_response({"ok": True}, status=201)

        async def recreate(req: web.Request) -> web.Response:
            b = await req.json()
            lc = lc_ref[0]
            ns, name = b.get("ns", "default"), b["pod"]
            lc.cluster.delete(ns, name, grace=0)
            await asyncio.sleep(float(b.get("gap_s", 0.0)))
            pod = lc.tenant(name, ns=ns, node=b.get("node", "node-0"))
            return web.json_response({"uid": pod["metadata"]["uid"]}, status=201)

        async def preemptions(req: web.Request) -> web.Response:
            from gpumounter_amd.cluster.pool import is_standby
            from gpumounter_amd.models.types import LABEL_APP, LABEL_APP_VALUE
            api = lc_ref[0].cluster
            kinds = {"standby": 0, "placeholder": 0, "other": 0}
            for v in api.victims:
                if is_standby(v):
                    kinds["standby"] += 1
                elif (v["metadata"].get("labels") or {}).get(LABEL_APP) == LABEL_APP_VALUE:
                    kinds["placeholder"] += 1
                else:
                    kinds["other"] += 1
            return web.json_response({"preemptions": api.preemptions, "victims": kinds})

        app.router.add_post("/_fake/faults", faults)
        app.router.add_post("/_fake/kubelet/restart", kubelet_restart)
        app.router.add_post("/_fake/recreate", recreate)
        app.router.add_post("/_fake/restart", restart)
        app.router.add_post("/_fake/tenant", tenant)
        app.router.add_post("/_fake/user", user)
        app.router.add_post("/_fake/worker", worker)
        app.router.add_get("/_fake/kubelet", kubelet)
        app.router.add_get("/_fake/preemptions", preemptions)
    return install


def _latency(name: str):
    """``zero`` (none), ``realistic`` (LatencyModel.realistic) or ``teardown`` (zero, except that
    the kubelet frees a deleted Pod's devices 50 ms after the DELETE: admission refusals)."""
    if name == "realistic":
        return LatencyModel.realistic()
    if name == "teardown":
        return LatencyModel(teardown_ms=50.0)
    return None


async def run(args) -> None:
    ref: list = [None]
    lc = LocalCluster(n_nodes=args.nodes, amdsmi_lib=args.amdsmi, cgroup_mode=args.cgroup,
                      latency=_latency(args.latency),
                      workdir=args.workdir, start_master=False, start_workers=False,
                      node_gpu_bdfs=[b for b in args.gpu_bdfs.split(",") if b] or None,
                      kubelet_limit_mode=args.kubelet_limit, gpu_api=args.gpu_api,
                      lazy_checkpoint=args.lazy_checkpoint,
                      app_hook=_hooks(ref), kernel_fs_dir=args.kernel_fs_dir)
    ref[0] = lc
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    await lc.start()
    # The stand-ins for the Go apiserver and kubelet should not add Python GC pauses of their
    # own to the latencies measured through them: freeze what start-up allocated, as the
    # daemons do (utils/runtime.py)
    runtime.tune_gc()
    runtime.watch_gc_pauses(5.0, log.get("fakes.controlplane"))
    info = {"api_url": lc.api_url, "pid": os.getpid(),
            "nodes": {name: {"kubelet_socket": h.kubelet.socket_path,
                             "kubelet_checkpoint": h.node.checkpoint_path,
                             "cgroup_root": h.node.cgroup_root,
                             "rootfs_root": h.node.rootfs_root,
                             "state_dir": h.node.state_dir, "host_dev": h.node.host_dev}
                      for name, h in lc.nodes.items()}}
    tmp = args.info + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(info, fh)
    os.replace(tmp, args.info)
    try:
        await stop.wait()
    finally:
        await lc.stop()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gpumounter_amd.fakes.controlplane")
    ap.add_argument("--workdir", required=True)
    ap.add_argument("--info", required=True)
    ap.add_argument("--nodes", type=int, default=1)
    ap.add_argument("--kernel-fs-dir", default="",
                    help="directory (a tmpfs) for the emulated cgroupfs and /dev trees")
    ap.add_argument("--amdsmi", default="mock")
    ap.add_argument("--cgroup", choices=("v1", "v2"), default="v2")
    ap.add_argument("--latency", choices=("zero", "realistic", "teardown"), default="zero")
    ap.add_argument("--kubelet-limit", choices=("enforce", "count"), default="enforce",
                    help="PodResources limiter (100 qps, burst 10): reject over-budget calls "
                         "with RESOURCE_EXHAUSTED, or serve them and only count them")
    ap.add_argument("--gpu-bdfs", default="", help="comma-separated: the node's GPUs (default all)")
    ap.add_argument("--lazy-checkpoint", action="store_true",
                    help="the device manager keeps a deleted Pod in its checkpoint until the "
                         "next Allocate, as a real kubelet does")
    ap.add_argument("--gpu-api", choices=("device-plugin", "dra"), default="device-plugin",
                    help="dra: the GPUs are published in ResourceSlices (fakes/dra.py)")
    args = ap.parse_args(argv)
    log.setup("WARNING", json_format=False)
    asyncio.run(run(args))
    return 0


if __name__ == "__main__":
    sys.exit(main())
