"""Tenant-visible side effects of attach/detach: core/v1 Events and a devices annotation.

The reference only logs (reference: pkg/server/gpu-mount/server.go:81-95). Here every successful
attach/detach, forced kill and reconciler revocation becomes an Event on the tenant pod, so
``kubectl describe pod`` shows what happened. With ``annotate_tenant`` the pod also carries
``gpumounter.amd.com/devices`` = the PCI BDFs it currently holds. A downward-API volume
projects that into the container, where it updates without a restart.

Neither is on the request path: sends are queued and flushed once the worker has had no
attach/detach in flight for ``notify_idle_ms`` (so the apiserver round trips never share the event
loop with a request), or after ``notify_max_delay_ms`` under sustained load. Identical Events
queued meanwhile (same Pod, reason, message and type — a Pod attached and detached in a loop)
are sent once with their ``count``, as client-go's event correlator aggregates them, so a flush
under sustained load is a handful of requests, not one per operation. Failures are logged,
never surfaced.
"""
from __future__ import annotations

import asyncio
import contextlib
import datetime
from typing import Awaitable, Callable, Dict, List, Optional, Sequence, Set, Tuple

from gpumounter_amd.models import pod as podu
from gpumounter_amd.models.device import AmdGpu
from gpumounter_amd.utils import calls, log

_log = log.get("worker.notify")
ANN_DEVICES = "gpumounter.amd.com/devices"


class Notifier:
    def __init__(self, cfg, kube) -> None:
        self.cfg = cfg
        self.kube = kube
        self._tasks: Set[asyncio.Task] = set()
        # (coalescing key or None, send): for a key only the newest send survives a flush
        self._queue: List[Tuple[Optional[tuple], Callable[[], Awaitable[None]]]] = []
        self._flusher: Optional[asyncio.Task] = None
        self._inflight = 0
        self._idle = asyncio.Event()
        self._idle.set()
        self.sent = 0
        # coalescing key → [first timestamp, count] of Events queued and not yet sent
        self._ev_pending: Dict[tuple, list] = {}

    @contextlib.contextmanager
    def operation(self):
        """Bracket one attach/detach: queued notifications wait until none is in flight."""
        self._inflight += 1
        self._idle.clear()
        try:
            yield
        finally:
            self._inflight -= 1
            if self._inflight == 0:
                self._idle.set()

    def _spawn(self, factory: Callable[[], Awaitable[None]], key: Optional[tuple] = None) -> None:
        self._queue.append((key, factory))
        self._kick()

    def _kick(self) -> None:
        if self._queue and (self._flusher is None or self._flusher.done()):
            t = self._flusher = asyncio.ensure_future(self._flush())
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)

    async def _wait_idle(self) -> None:
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.cfg.notify_max_delay_ms / 1e3
        quiet = self.cfg.notify_idle_ms / 1e3
        while True:
            if self._inflight == 0:
                await asyncio.sleep(quiet)        # lets the finished RPC's reply go out first
                if self._inflight == 0:
                    return
            left = deadline - loop.time()
            if left <= 0:
                return
            # asyncio.wait, not wait_for: on Python 3.10 wait_for can swallow a cancellation
            # that arrives as the inner wait completes (the waiter's task then never stops)
            waiter = asyncio.ensure_future(self._idle.wait())
            try:
                done, _ = await asyncio.wait({waiter}, timeout=left)
            finally:
                if not waiter.done():
                    waiter.cancel()
            if not done:
                return

    async def quiet(self) -> None:
        """Until no attach/detach has been in flight for ``notify_idle_ms`` (at most
        ``notify_max_delay_ms``): background work that should not share the event loop with a
        request (Events, the warm pool's refill) waits for this."""
        await self._wait_idle()

    async def _flush(self) -> None:
        calls.mark_background()
        while self._queue:
            await self._wait_idle()
            batch, self._queue = self._queue, []
            latest: Dict[tuple, int] = {k: i for i, (k, _) in enumerate(batch) if k is not None}
            sends = [f() for i, (k, f) in enumerate(batch) if k is None or latest[k] == i]
            await asyncio.gather(*sends, return_exceptions=True)

    async def drain(self) -> None:
        """Wait for pending notifications (tests, shutdown)."""
        while self._tasks or self._queue:
            self._kick()
            await asyncio.gather(*list(self._tasks), return_exceptions=True)

    async def stop(self) -> None:
        self._queue.clear()
        self._ev_pending.clear()
        for t in list(self._tasks):
            t.cancel()

    # ------------------------------------------------------------------------ events
    def event(self, pod: dict, reason: str, message: str, warning: bool = False) -> None:
        if not self.cfg.emit_events:
            return
        now = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        ns, name = podu.ns_of(pod), podu.name_of(pod)
        key = ("event", ns, name, podu.uid_of(pod), reason, message[:1024], warning)
        agg = self._ev_pending.get(key)
        if agg is not None:
            agg[1] += 1                     # queued already: counted into that one
            agg[2] = now
            return
        self._ev_pending[key] = agg = [now, 1, now]
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f"{name}.", "namespace": ns},
              "involvedObject": {"apiVersion": "v1", "kind": "Pod", "namespace": ns,
                                 "name": name, "uid": podu.uid_of(pod)},
              "reason": reason, "message": message[:1024],
              "type": "Warning" if warning else "Normal",
              "source": {"component": "gpumounter-worker", "host": self.cfg.node_name},
              "reportingComponent": "gpumounter-amd/worker",
              "reportingInstance": self.cfg.node_name}

        async def send():
            self._ev_pending.pop(key, None)
            ev.update(firstTimestamp=agg[0], lastTimestamp=agg[2], count=agg[1])
            try:
                await self.kube.create_event(ns, ev)
                self.sent += 1
            except Exception as e:  # noqa: BLE001
                _log.debug("event %s on %s/%s not recorded: %s", reason, ns, name, e)
        self._spawn(send)

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
        self._spawn(send, key=("annotate", podu.ns_of(pod), podu.name_of(pod)))

    # ------------------------------------------------------------------------ helpers
    @staticmethod
    def describe(gs: Sequence[AmdGpu]) -> str:
        return ", ".join(f"{g.bdf} (renderD{g.render_minor})" for g in gs)

    @staticmethod
    def _by(user: str) -> str:
        return f" (requested by {user})" if user else ""

    def attached(self, pod: dict, new: Sequence[AmdGpu], holding: Sequence[AmdGpu],
                 mode: str, by: str = "") -> None:
        self.event(pod, "GPUAttached",
                   f"hot-mounted {len(new)} GPU(s) ({mode}): {self.describe(new)}{self._by(by)}")
        self.annotate(pod, holding)

    def detached(self, pod: dict, removed: Sequence[AmdGpu], holding: Sequence[AmdGpu],
                 killed: Sequence[int], by: str = "") -> None:
        self.event(pod, "GPUDetached",
                   f"removed {len(removed)} GPU(s): {self.describe(removed)}{self._by(by)}")
        if killed:
            self.event(pod, "GPUProcessesTerminated",
                       f"force-removed GPUs were in use; signalled PIDs {list(killed)}",
                       warning=True)
        self.annotate(pod, holding)
