"""Fake kubelet: PodResources server (v1 + v1alpha1) and, optionally, a device manager.

Backed by a :class:`FakeNode`'s device-plugin ledger, so the worker reads allocations through the
same gRPC surface it uses against a real kubelet (reference: pkg/util/gpu/collector/
collector.go:165-194 dials ``/var/lib/kubelet/pod-resources/kubelet.sock``).

With ``plugin_dir`` it also serves ``v1beta1.Registration`` on ``<plugin_dir>/kubelet.sock``; a
plugin that registers gets the kubelet device-manager treatment over its own socket
(GetDevicePluginOptions, a ListAndWatch stream for health, GetPreferredAllocation when
advertised, then Allocate at admission).
"""
from __future__ import annotations

import asyncio
import os
from typing import Dict, List, Optional, Tuple

import grpc

from gpumounter_amd.api import deviceplugin as dp
from gpumounter_amd.api.podresources import V1, V1ALPHA1
from gpumounter_amd.fakes.node import FakeNode
from gpumounter_amd.utils.ratelimit import TokenBucket


class FakeKubelet:
    def __init__(self, node: FakeNode, socket_path: str, serve_v1: bool = True,
                 serve_v1alpha1: bool = True, plugin_dir: str = "",
                 rate_limit: Optional[Tuple[float, int]] = (100.0, 10),
                 limit_mode: str = "enforce") -> None:
        self.node = node
        # the kubelet's PodResources limiter (pkg/kubelet/apis/podresources: DefaultQPS 100,
        # DefaultBurstTokens 10): over budget → RESOURCE_EXHAUSTED "rejected by rate limit".
        # limit_mode "count" serves every call but counts the ones a limited kubelet would
        # reject (calls["over_limit"]): how the emulated reference, which has no retry, is
        # measured without failing (it would fail against a limited kubelet).
        if limit_mode not in ("enforce", "count"):
            raise ValueError(f"limit_mode {limit_mode!r}")
        self.limiter = TokenBucket(*rate_limit) if rate_limit else None
        self.limit_mode = limit_mode
        self.socket_path = socket_path
        self.serve_v1 = serve_v1
        self.serve_v1alpha1 = serve_v1alpha1
        self.plugin_dir = plugin_dir
        self.server = None
        self.reg_server = None
        self.calls = {"List": 0, "GetAllocatableResources": 0, "Get": 0, "Register": 0,
                      "rejected": 0, "over_limit": 0}
        # device manager state
        self.plugin_endpoint = ""
        self.plugin_options = None
        self.plugin_devices: Dict[str, str] = {}   # device id → health
        self._plugin_ch: Optional[grpc.aio.Channel] = None
        self._law_task: Optional[asyncio.Task] = None
        self._alloc_lock = asyncio.Lock()
        self.preferred_log: List[List[str]] = []

    # ------------------------------------------------------------------------ device manager
    async def _register(self, request, context):
        self.calls["Register"] += 1
        if request.version != dp.VERSION or request.resource_name != self.node.resource:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, "unsupported registration")
        await self._drop_plugin()
        self.plugin_endpoint = request.endpoint
        self._plugin_ch = grpc.aio.insecure_channel(
            f"unix://{os.path.join(self.plugin_dir, request.endpoint)}")
        opts = self._plugin_ch.unary_unary(dp.GET_OPTIONS, dp.Empty.SerializeToString,
                                           dp.DevicePluginOptions.FromString)
        self.plugin_options = await opts(dp.Empty(), timeout=5)
        first = asyncio.Event()
        self._law_task = asyncio.ensure_future(self._list_and_watch(first))
        await asyncio.wait_for(first.wait(), 5)
        self.node.plugin = self
        return dp.Empty()

    async def _list_and_watch(self, first: asyncio.Event) -> None:
        law = self._plugin_ch.unary_stream(dp.LIST_AND_WATCH, dp.Empty.SerializeToString,
                                           dp.ListAndWatchResponse.FromString)
        try:
            async for resp in law(dp.Empty()):
                self.plugin_devices = {d.ID: d.health for d in resp.devices}
                self.node.unhealthy = {i for i, h in self.plugin_devices.items()
                                       if h != dp.HEALTHY}
                first.set()
        except (grpc.aio.AioRpcError, asyncio.CancelledError):
            pass

    async def _drop_plugin(self) -> None:
        self.node.plugin = None
        if self._law_task is not None:
            self._law_task.cancel()
            self._law_task = None
        if self._plugin_ch is not None:
            await self._plugin_ch.close()
            self._plugin_ch = None

    async def plugin_allocate(self, ns: str, pod: str, container: str, n: int,
                              uid: str = "") -> Optional[List[str]]:
        """Device-manager admission: healthy free devices → GetPreferredAllocation → Allocate."""
        async with self._alloc_lock:
            free = [d for d in self.node.free_ids() if d not in self.node.unhealthy
                    and d in self.plugin_devices]
            if len(free) < n:
                return None
            ids = free[:n]
            if self.plugin_options.get_preferred_allocation_available and len(free) > n:
                pref = self._plugin_ch.unary_unary(
                    dp.GET_PREFERRED, dp.PreferredAllocationRequest.SerializeToString,
                    dp.PreferredAllocationResponse.FromString)
                req = dp.PreferredAllocationRequest()
                req.container_requests.add(available_deviceIDs=free, allocation_size=n)
                resp = await pref(req, timeout=5)
                got = list(resp.container_responses[0].deviceIDs)
                if len(got) == n and set(got) <= set(free):   # kubelet validates the same way
                    ids = got
                self.preferred_log.append(ids)
            alloc = self._plugin_ch.unary_unary(dp.ALLOCATE, dp.AllocateRequest.SerializeToString,
                                                dp.AllocateResponse.FromString)
            req = dp.AllocateRequest()
            req.container_requests.add(devices_ids=ids)
            await alloc(req, timeout=5)
            return ids if self.node.record(ns, pod, container, ids, uid=uid) else None

    def _fill(self, api, resp, only=None):
        for (ns, pod), containers in sorted(self.node.ledger().items()):
            if only and (ns, pod) != only:
                continue
            pr = resp.pod_resources.add(name=pod, namespace=ns) if only is None else resp
            for cname, res in sorted(containers.items()):
                c = pr.containers.add(name=cname)
                for rname, ids in sorted(res.items()):
                    d = c.devices.add(resource_name=rname, device_ids=ids)
                    if api is V1:
                        numas = sorted({self.node.numa_of(i) for i in ids} - {-1})
                        for n in numas:
                            d.topology.nodes.add(ID=n)
        return resp

    async def _police(self, context) -> None:
        if self.limiter is not None and not self.limiter.allow():
            self.calls["over_limit"] += 1
            if self.limit_mode == "count":
                return
            self.calls["rejected"] += 1
            await context.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, "rejected by rate limit")

    def _list(self, api):
        async def handler(request, context):
            await self._police(context)
            self.calls["List"] += 1
            return self._fill(api, api.ListPodResourcesResponse())
        return handler

    async def _allocatable(self, request, context):
        await self._police(context)
        self.calls["GetAllocatableResources"] += 1
        resp = V1.AllocatableResourcesResponse()
        for g in self.node.gpus:
            d = resp.devices.add(resource_name=self.node.resource,
                                 device_ids=[self.node.device_id(g)])
            if g.numa_node >= 0:
                d.topology.nodes.add(ID=g.numa_node)
        return resp

    async def _get(self, request, context):
        await self._police(context)
        self.calls["Get"] += 1
        resp = V1.GetPodResourcesResponse()
        key = (request.pod_namespace, request.pod_name)
        resp.pod_resources.name = request.pod_name
        resp.pod_resources.namespace = request.pod_namespace
        if key in self.node.ledger():
            self._fill(V1, resp.pod_resources, only=key)
        return resp

    async def start(self) -> None:
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        os.makedirs(os.path.dirname(self.socket_path), exist_ok=True)
        self.server = grpc.aio.server()
        handlers = []
        if self.serve_v1:
            handlers.append(grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
                "List": grpc.unary_unary_rpc_method_handler(
                    self._list(V1), V1.ListPodResourcesRequest.FromString,
                    lambda m: m.SerializeToString()),
                "GetAllocatableResources": grpc.unary_unary_rpc_method_handler(
                    self._allocatable, V1.AllocatableResourcesRequest.FromString,
                    lambda m: m.SerializeToString()),
                "Get": grpc.unary_unary_rpc_method_handler(
                    self._get, V1.GetPodResourcesRequest.FromString,
                    lambda m: m.SerializeToString()),
            }))
        if self.serve_v1alpha1:
            handlers.append(grpc.method_handlers_generic_handler("v1alpha1.PodResourcesLister", {
                "List": grpc.unary_unary_rpc_method_handler(
                    self._list(V1ALPHA1), V1ALPHA1.ListPodResourcesRequest.FromString,
                    lambda m: m.SerializeToString()),
            }))
        self.server.add_generic_rpc_handlers(tuple(handlers))
        self.server.add_insecure_port(f"unix://{self.socket_path}")
        await self.server.start()
        if self.plugin_dir:
            await self.start_registration()

    async def start_registration(self) -> None:
        os.makedirs(self.plugin_dir, exist_ok=True)
        path = os.path.join(self.plugin_dir, dp.KUBELET_SOCKET)
        if os.path.exists(path):
            os.unlink(path)
        self.reg_server = grpc.aio.server()
        self.reg_server.add_generic_rpc_handlers([grpc.method_handlers_generic_handler(
            "v1beta1.Registration", {"Register": grpc.unary_unary_rpc_method_handler(
                self._register, dp.RegisterRequest.FromString, dp.Empty.SerializeToString)})])
        self.reg_server.add_insecure_port(f"unix://{path}")
        await self.reg_server.start()

    async def restart(self) -> None:
        """Kubelet restart: forget plugins and wipe the socket directory (as the real one)."""
        await self._drop_plugin()
        if self.reg_server is not None:
            await self.reg_server.stop(0)
        for f in os.listdir(self.plugin_dir):
            if f.endswith(".sock"):
                os.unlink(os.path.join(self.plugin_dir, f))
        await self.start_registration()

    async def stop(self) -> None:
        await self._drop_plugin()
        if self.reg_server is not None:
            await self.reg_server.stop(0)
            self.reg_server = None
        if self.server is not None:
            await self.server.stop(0)
            self.server = None
