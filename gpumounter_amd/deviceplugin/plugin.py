"""``amd.com/gpu`` device plugin with placement steering.

The reference cannot choose which GPUs its slave pods get: NVIDIA's device plugin picks them
(reference: pkg/util/gpu/allocator/allocator.go:214-231, no topology input). When
gpumounter-amd also serves the resource (``GM_DEVICE_PLUGIN=1``, replacing the ROCm plugin on
the node), it controls that choice:

* ``ListAndWatch`` advertises every GPU of the amdsmi inventory by PCI BDF (the ID the ROCm
  plugin uses, so PodResources joins stay the same) with its NUMA node as topology hint, and
  re-sends the list when amdsmi health changes;
* ``GetPreferredAllocation`` first consumes an *intent* the worker registered right before it
  created the placeholder (the xGMI/NUMA-chosen set), otherwise applies the same topology policy
  to whatever is available — so ordinary ``amd.com/gpu`` pods get hive/NUMA-packed sets too;
* ``Allocate`` returns ``/dev/kfd`` + ``/dev/dri/renderD*`` + ``/dev/dri/card*`` device specs
  (``inject_devices=False`` for CPU-only clusters such as kind with the mock inventory);
* the plugin re-registers when the kubelet restarts (it wipes the socket directory).

Correctness never depends on the steering: the kubelet ledger stays authoritative and the
worker mounts whatever was allocated.
"""
from __future__ import annotations

import asyncio
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import grpc

from gpumounter_amd.api import deviceplugin as dp
from gpumounter_amd.hw import topology
from gpumounter_amd.models.device import AmdGpu, normalize_device_id
from gpumounter_amd.utils import log

_log = log.get("deviceplugin")


@dataclass
class Intent:
    ids: tuple
    created: float
    token: str


class AmdGpuDevicePlugin:
    def __init__(self, inv, resource: str = "amd.com/gpu",
                 plugin_dir: str = dp.DEVICE_PLUGIN_DIR, socket_name: str = "gpumounter-amd.sock",
                 inject_devices: bool = True, health_period_s: float = 5.0,
                 policy: str = "xgmi", intent_ttl_s: float = 60.0, metrics=None) -> None:
        self.inv = inv
        self.resource = resource
        self.plugin_dir = plugin_dir
        self.socket_name = socket_name
        self.inject_devices = inject_devices
        self.health_period_s = health_period_s
        self.policy = policy
        self.intent_ttl_s = intent_ttl_s
        self.intents: List[Intent] = []
        self.health: Dict[int, bool] = {g.index: True for g in inv.gpus()}
        self.server: Optional[grpc.aio.Server] = None
        self.registered = 0
        self.calls: Dict[str, int] = {"Allocate": 0, "GetPreferredAllocation": 0,
                                      "ListAndWatch": 0, "steered": 0}
        self.metrics = metrics
        self._subs: set = set()   # one event per open ListAndWatch stream
        self._tasks: List[asyncio.Task] = []
        self._sock_ino = 0
        self._stopping = False

    def _count(self, rpc: str) -> None:
        self.calls[rpc] += 1
        if self.metrics is not None:
            self.metrics.plugin_rpcs.labels(rpc=rpc).inc()

    # ------------------------------------------------------------------------ identity
    @property
    def socket_path(self) -> str:
        return os.path.join(self.plugin_dir, self.socket_name)

    @staticmethod
    def device_id(g: AmdGpu) -> str:
        return g.bdf

    def _gpu(self, device_id: str) -> Optional[AmdGpu]:
        return self.inv.by_key().get(normalize_device_id(device_id))

    def devices(self) -> List["dp.Device"]:
        out = []
        for g in self.inv.gpus():
            d = dp.Device(ID=self.device_id(g),
                          health=dp.HEALTHY if self.health.get(g.index, True) else dp.UNHEALTHY)
            if g.numa_node >= 0:
                d.topology.nodes.add(ID=g.numa_node)
            out.append(d)
        return out

    # ------------------------------------------------------------------------ steering
    def intend(self, ids: Sequence[str], token: str = "") -> None:
        """The worker is about to create a placeholder that should get exactly ``ids``."""
        now = time.monotonic()
        self.intents = [i for i in self.intents if now - i.created < self.intent_ttl_s]
        self.intents.append(Intent(tuple(normalize_device_id(d) for d in ids), now, token))

    def withdraw(self, token: str) -> None:
        self.intents = [i for i in self.intents if i.token != token]

    def prefer(self, available: Sequence[str], must: Sequence[str], size: int) -> List[str]:
        avail = {normalize_device_id(d): d for d in available}
        must_n = [normalize_device_id(d) for d in must]
        for i, it in enumerate(self.intents):
            if len(it.ids) == size and all(d in avail for d in it.ids) and \
                    set(must_n) <= set(it.ids):
                del self.intents[i]
                self._count("steered")
                return [avail[d] for d in it.ids]
        cands = [g for d in avail if d not in must_n for g in [self._gpu(d)] if g is not None
                 and self.health.get(g.index, True)]
        attached = [g for d in must_n for g in [self._gpu(d)] if g is not None]
        plc = topology.choose(cands, size - len(must_n), self.inv.links(), attached=attached,
                              policy=self.policy)
        if plc is None:
            return list(must) + [d for d in available if normalize_device_id(d) not in must_n][
                :max(size - len(must_n), 0)]
        by_index = {g.index: g for g in cands}
        return list(must) + [avail[normalize_device_id(self.device_id(by_index[i]))]
                             for i in plc.chosen]

    # ------------------------------------------------------------------------ RPCs
    async def _options(self, req, ctx):
        return dp.DevicePluginOptions(get_preferred_allocation_available=True)

    def _notify(self) -> None:
        for ev in list(self._subs):
            ev.set()

    async def _list_and_watch(self, req, ctx):
        self._count("ListAndWatch")
        ev = asyncio.Event()
        self._subs.add(ev)
        try:
            while not self._stopping:
                ev.clear()
                yield dp.ListAndWatchResponse(devices=self.devices())
                await ev.wait()
        finally:
            self._subs.discard(ev)

    async def _preferred(self, req, ctx):
        self._count("GetPreferredAllocation")
        resp = dp.PreferredAllocationResponse()
        for cr in req.container_requests:
            ids = self.prefer(list(cr.available_deviceIDs), list(cr.must_include_deviceIDs),
                              cr.allocation_size)
            resp.container_responses.add(deviceIDs=ids)
        return resp

    async def _allocate(self, req, ctx):
        self._count("Allocate")
        resp = dp.AllocateResponse()
        for cr in req.container_requests:
            c = resp.container_responses.add()
            gs = []
            for d in cr.devices_ids:
                g = self._gpu(d)
                if g is None:
                    await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown device {d}")
                gs.append(g)
            if not self.inject_devices:
                continue
            c.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            for g in gs:
                for n in g.device_nodes():
                    c.devices.add(container_path=n.path, host_path=n.path, permissions="rw")
        return resp

    async def _pre_start(self, req, ctx):
        return dp.PreStartContainerResponse()

    # ------------------------------------------------------------------------ lifecycle
    async def start(self, register: bool = True) -> None:
        os.makedirs(self.plugin_dir, exist_ok=True)
        await self._serve()
        if register:
            await self.register()
        self._tasks.append(asyncio.ensure_future(self._health_loop()))
        self._tasks.append(asyncio.ensure_future(self._kubelet_restart_loop()))

    async def _serve(self) -> None:
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        server = grpc.aio.server()
        server.add_generic_rpc_handlers([grpc.method_handlers_generic_handler(
            "v1beta1.DevicePlugin", {
                "GetDevicePluginOptions": grpc.unary_unary_rpc_method_handler(
                    self._options, dp.Empty.FromString, dp.DevicePluginOptions.SerializeToString),
                "ListAndWatch": grpc.unary_stream_rpc_method_handler(
                    self._list_and_watch, dp.Empty.FromString,
                    dp.ListAndWatchResponse.SerializeToString),
                "GetPreferredAllocation": grpc.unary_unary_rpc_method_handler(
                    self._preferred, dp.PreferredAllocationRequest.FromString,
                    dp.PreferredAllocationResponse.SerializeToString),
                "Allocate": grpc.unary_unary_rpc_method_handler(
                    self._allocate, dp.AllocateRequest.FromString,
                    dp.AllocateResponse.SerializeToString),
                "PreStartContainer": grpc.unary_unary_rpc_method_handler(
                    self._pre_start, dp.PreStartContainerRequest.FromString,
                    dp.PreStartContainerResponse.SerializeToString),
            })])
        server.add_insecure_port(f"unix://{self.socket_path}")
        await server.start()
        self.server = server
        self._sock_ino = os.stat(self.socket_path).st_ino

    async def register(self) -> None:
        kubelet = os.path.join(self.plugin_dir, dp.KUBELET_SOCKET)
        async with grpc.aio.insecure_channel(f"unix://{kubelet}") as ch:
            stub = ch.unary_unary(dp.REGISTER, request_serializer=dp.RegisterRequest.SerializeToString,
                                  response_deserializer=dp.Empty.FromString)
            await stub(dp.RegisterRequest(
                version=dp.VERSION, endpoint=self.socket_name, resource_name=self.resource,
                options=dp.DevicePluginOptions(get_preferred_allocation_available=True)),
                timeout=10)
        self.registered += 1
        _log.info("registered %s with the kubelet (%d devices)", self.resource,
                  len(self.health))

    async def _health_loop(self) -> None:
        while not self._stopping:
            await asyncio.sleep(self.health_period_s)
            try:
                h = await asyncio.get_running_loop().run_in_executor(None, self.inv.healthy)
            except Exception as e:  # noqa: BLE001
                _log.warning("health probe failed: %s", e)
                continue
            if h != self.health:
                _log.warning("GPU health changed: %s", {i: v for i, v in h.items()
                                                         if self.health.get(i) != v})
                self.health = h
                self._notify()

    async def _kubelet_restart_loop(self) -> None:
        """A restarting kubelet deletes every socket in the directory: serve again, re-register."""
        while not self._stopping:
            await asyncio.sleep(1.0)
            try:
                ino = os.stat(self.socket_path).st_ino
            except FileNotFoundError:
                ino = 0
            if ino == self._sock_ino:
                continue
            _log.warning("device-plugin socket gone (kubelet restart?); re-registering")
            try:
                if self.server is not None:
                    await self.server.stop(0)
                await self._serve()
                await self.register()
            except Exception as e:  # noqa: BLE001
                _log.error("re-register failed: %s", e)

    def set_health(self, index: int, ok: bool) -> None:
        """Test/operator hook: force a device's health (e.g. drained for maintenance)."""
        self.health[index] = ok
        self._notify()

    async def stop(self) -> None:
        self._stopping = True
        self._notify()
        for t in self._tasks:
            t.cancel()
        if self.server is not None:
            await self.server.stop(0.2)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
