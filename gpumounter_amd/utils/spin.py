"""Keep an asyncio loop polling while a latency-critical request is in flight.

An attach is a chain of short waits: the gRPC request reaching the worker, each apiserver
reply, the watch event of the admitted placeholder, the gRPC response reaching the master.
Each wait ends with a wake-up of a thread that blocked in ``epoll_wait``. The loop thread is
woken by the socket; a grpc.aio completion is first handed by grpc's poller thread through a
socket pair. On a loaded or virtualised host one such wake-up costs tens of microseconds, and
the attach pays for a dozen. The bench's box calibration measures this as
``pingpong_after_idle_us`` (``gpumounter_amd/utils/calib.py``).

:class:`LoopSpinner` removes the loop thread's share of those wake-ups. While at least one
request holds it, and for ``tail_us`` after the last one lets go (the response is still being
written), a callback re-schedules itself on every loop iteration. The loop then polls with a
zero timeout instead of blocking. The spin is capped at ``max_ms`` per stretch, so a long
operation (a force removal waiting for processes to exit) falls back to blocking waits.
``epoll_wait(0)`` releases the GIL like the blocking call, so other threads are not starved.

Config: ``loop_spin_us`` (0 = off), ``loop_spin_max_ms``.
"""
from __future__ import annotations

import asyncio
import contextlib
import time
from typing import Optional


class LoopSpinner:
    def __init__(self, tail_us: float, max_ms: float = 20.0) -> None:
        self.tail_s = max(tail_us, 0.0) / 1e6
        self.max_s = max(max_ms, 0.0) / 1e3
        self.enabled = self.tail_s > 0 and self.max_s > 0
        self._held = 0
        self._until = 0.0
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._spinning = False
        self.ticks = 0          # loop iterations spent polling (for tests and metrics)

    def _tick(self) -> None:
        if time.perf_counter() < self._until:
            self.ticks += 1
            self._loop.call_soon(self._tick)
        else:
            self._spinning = False

    def _start(self) -> None:
        if not self._spinning:
            self._spinning = True
            self._loop = asyncio.get_running_loop()
            self._loop.call_soon(self._tick)

    @contextlib.contextmanager
    def hold(self):
        """Spin while the body runs (at most ``max_ms`` from its start) and ``tail_us`` after."""
        if not self.enabled:
            yield
            return
        self._held += 1
        self._until = max(self._until, time.perf_counter() + self.max_s)
        self._start()
        try:
            yield
        finally:
            self._held -= 1
            if self._held == 0:
                self._until = min(self._until, time.perf_counter() + self.tail_s)
