"""Fake kubelet PodResources server (v1 + v1alpha1) on a unix socket.

Backed by a :class:`FakeNode`'s device-plugin ledger, so the worker reads allocations through the
same gRPC surface it uses against a real kubelet (reference: pkg/util/gpu/collector/
collector.go:165-194 dials ``/var/lib/kubelet/pod-resources/kubelet.sock``).
"""
from __future__ import annotations

import os

import grpc

from gpumounter_amd.api.podresources import V1, V1ALPHA1
from gpumounter_amd.fakes.node import FakeNode


class FakeKubelet:
    def __init__(self, node: FakeNode, socket_path: str, serve_v1: bool = True,
                 serve_v1alpha1: bool = True) -> None:
        self.node = node
        self.socket_path = socket_path
        self.serve_v1 = serve_v1
        self.serve_v1alpha1 = serve_v1alpha1
        self.server = None
        self.calls = {"List": 0, "GetAllocatableResources": 0, "Get": 0}

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

    def _list(self, api):
        async def handler(request, context):
            self.calls["List"] += 1
            return self._fill(api, api.ListPodResourcesResponse())
        return handler

    async def _allocatable(self, request, context):
        self.calls["GetAllocatableResources"] += 1
        resp = V1.AllocatableResourcesResponse()
        for g in self.node.gpus:
            d = resp.devices.add(resource_name=self.node.resource,
                                 device_ids=[self.node.device_id(g)])
            if g.numa_node >= 0:
                d.topology.nodes.add(ID=g.numa_node)
        return resp

    async def _get(self, request, context):
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

    async def stop(self) -> None:
        if self.server is not None:
            await self.server.stop(0)
            self.server = None
