"""Tenant-visible side effects of attach/detach: core/v1 Events and a devices annotation.

The reference only logs (reference: pkg/server/gpu-mount/server.go:81-95). Here every successful
attach/detach, forced kill and reconciler revocation becomes an Event on the tenant pod, so
``kubectl describe pod`` shows what happened. With ``annotate_tenant`` the pod also carries
``gpumounter.amd.com/devices`` = the PCI BDFs it currently holds. A downward-API volume
projects that into the container, where it updates without a restart.

Both run after the RPC has answered (fire-and-forget tasks); failures are logged, never surfaced.
"""
from __future__ import annotations

import asyncio
import datetime
from typing import Sequence, Set

from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.device import AmdGpu
from gpumounter_amd.utils import log

_log = log.get("worker.notify")
ANN_DEVICES = "gpumounter.amd.com/devices"


class Notifier:
    def __init__(self, cfg, kube) -> None:
        self.cfg = cfg
        self.kube = kube
        self._tasks: Set[asyncio.Task] = set()
        self.sent = 0

    def _spawn(self, coro) -> None:
        t = asyncio.ensure_future(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    async def drain(self) -> None:
        """Wait for pending notifications (tests, shutdown)."""
        while self._tasks:
            await asyncio.gather(*list(self._tasks), return_exceptions=True)

    async def stop(self) -> None:
        for t in list(self._tasks):
            t.cancel()

    # ------------------------------------------------------------------------ events
    def event(self, pod: dict, reason: str, message: str, warning: bool = False) -> None:
        if not self.cfg.emit_events:
            return
        now = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        ns, name = podu.ns_of(pod), podu.name_of(pod)
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f"{name}.", "namespace": ns},
              "involvedObject": {"apiVersion": "v1", "kind": "Pod", "namespace": ns,
                                 "name": name, "uid": podu.uid_of(pod)},
              "reason": reason, "message": message[:1024],
              "type": "Warning" if warning else "Normal",
              "source": {"component": "gpumounter-worker", "host": self.cfg.node_name},
              "reportingComponent": "gpumounter-amd/worker",
              "reportingInstance": self.cfg.node_name,
              "firstTimestamp": now, "lastTimestamp": now, "count": 1}

        async def send():
            try:
                await self.kube.create_event(ns, ev)
                self.sent += 1
            except Exception as e:  # noqa: BLE001
                _log.debug("event %s on %s/%s not recorded: %s", reason, ns, name, e)
        self._spawn(send())

    # ------------------------------------------------------------------------ annotation
    def annotate(self, pod: dict, holding: Sequence[AmdGpu]) -> None:
        if not self.cfg.annotate_tenant:
            return
        value = ",".join(g.bdf for g in sorted(holding, key=lambda g: g.index)) or None
        patch = {"metadata": {"annotations": {ANN_DEVICES: value}}}

        async def send():
            try:
                await self.kube.patch_pod(podu.ns_of(pod), podu.name_of(pod), patch)
            except Exception as e:  # noqa: BLE001
                _log.debug("annotate %s/%s failed: %s", podu.ns_of(pod), podu.name_of(pod), e)
        self._spawn(send())

    # ------------------------------------------------------------------------ helpers
    @staticmethod
    def describe(gs: Sequence[AmdGpu]) -> str:
        return ", ".join(f"{g.bdf} (renderD{g.render_minor})" for g in gs)

    def attached(self, pod: dict, new: Sequence[AmdGpu], holding: Sequence[AmdGpu],
                 mode: str) -> None:
        self.event(pod, "GPUAttached",
                   f"hot-mounted {len(new)} GPU(s) ({mode}): {self.describe(new)}")
        self.annotate(pod, holding)

    def detached(self, pod: dict, removed: Sequence[AmdGpu], holding: Sequence[AmdGpu],
                 killed: Sequence[int]) -> None:
        self.event(pod, "GPUDetached",
                   f"removed {len(removed)} GPU(s): {self.describe(removed)}")
        if killed:
            self.event(pod, "GPUProcessesTerminated",
                       f"force-removed GPUs were in use; signalled PIDs {list(killed)}",
                       warning=True)
        self.annotate(pod, holding)
