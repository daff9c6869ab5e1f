"""Token bucket, shared by the kubelet PodResources client (pacing) and the fake kubelet (policing).

Kubelets rate-limit their PodResources gRPC server with a token bucket — 100 requests/s, burst
10 by default — and answer the excess with ``RESOURCE_EXHAUSTED`` ("rejected by rate limit"). The
reference makes one List per query and never sees this (reference:
pkg/util/gpu/collector/collector.go:90-138); a controller that reads the ledger on the attach path
must pace itself under that budget and treat a rejection as "retry later", not as a failure.
"""
from __future__ import annotations

import asyncio
import time
from typing import Optional


class TokenBucket:
    def __init__(self, qps: float, burst: int, clock=time.monotonic) -> None:
        if qps <= 0 or burst <= 0:
            raise ValueError("qps and burst must be positive")
        self.qps = float(qps)
        self.burst = int(burst)
        self._clock = clock
        self._tokens = float(burst)
        self._t = clock()
        self._lock: Optional[asyncio.Lock] = None
        self._loop = None
        self.allowed = 0
        self.rejected = 0

    def _refill(self) -> None:
        now = self._clock()
        self._tokens = min(self.burst, self._tokens + (now - self._t) * self.qps)
        self._t = now

    def allow(self) -> bool:
        """Take a token if one is available (server side: reject otherwise)."""
        self._refill()
        if self._tokens >= 1.0:
            self._tokens -= 1.0
            self.allowed += 1
            return True
        self.rejected += 1
        return False

    def wait_time(self) -> float:
        self._refill()
        return 0.0 if self._tokens >= 1.0 else (1.0 - self._tokens) / self.qps

    async def acquire(self) -> float:
        """Wait for a token (client side: pace instead of being rejected). Returns the wait."""
        loop = asyncio.get_running_loop()
        if self._lock is None or self._loop is not loop:
            self._lock, self._loop = asyncio.Lock(), loop
        waited = 0.0
        async with self._lock:       # FIFO: concurrent callers queue instead of racing
            while True:
                w = self.wait_time()
                if w <= 0:
                    self._tokens -= 1.0
                    self.allowed += 1
                    return waited
                await asyncio.sleep(w)
                waited += w
