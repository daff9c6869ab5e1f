"""Which control-plane calls an operation makes, and how many of them are serial.

Fake-cluster timings are sub-millisecond; on a real cluster every apiserver or kubelet round
trip costs a millisecond or more, so the number of round trips an attach waits for one after the
other is what carries over. Each process keeps a ring of its outbound calls (apiserver requests
from :class:`~gpumounter_amd.cluster.kube.KubeClient`, kubelet PodResources RPCs from
:class:`~gpumounter_amd.node.ledger.LedgerClient`, device-manager checkpoint reads) as
``(start, end, kind)`` on CLOCK_MONOTONIC, the same clock in every process of a host. The worker
and master serve it on their debug endpoints (``debug_endpoints``); ``bench.py`` reads it around
a few attaches and detaches and reports, per operation, the calls by kind and the **serial round
trips**: the longest chain of calls each of which started after the previous one ended (calls
sent together with ``gather`` count once).

The reference's attach (cmd/GPUMounter-master/main.go:52-96 → pkg/util/gpu/allocator/
allocator.go:40-99,189-282) is the baseline: GET pod, LIST workers, one create per slave pod in
sequence, then a poll of GETs per slave pod until Running, then a PodResources List per pod.
"""
from __future__ import annotations

import contextvars
import time
from collections import deque
from typing import Deque, Dict, Iterable, List, Tuple

Call = Tuple[float, float, str]
BACKGROUND = " (background)"

_RING: Deque[Call] = deque(maxlen=8192)
_BG: contextvars.ContextVar[bool] = contextvars.ContextVar("gm_calls_background", default=False)


def mark_background() -> None:
    """Called at the top of a background task (pool refill, Event flush, watch relists, the
    reconciler, lease timers): its calls, and those of tasks it starts, are logged with the
    suffix `` (background)`` — in an operation's window, but nothing the operation waits for."""
    _BG.set(True)


def record(kind: str, t0: float, t1: float) -> None:
    _RING.append((t0, t1, kind + BACKGROUND if _BG.get() else kind))


class span:
    """``with calls.span("apiserver POST pods"):`` around one outbound call."""

    __slots__ = ("kind", "t0")

    def __init__(self, kind: str) -> None:
        self.kind = kind

    def __enter__(self):
        self.t0 = time.monotonic()
        return self

    def __exit__(self, *exc) -> None:
        record(self.kind, self.t0, time.monotonic())


def since(t0: float, t1: float = float("inf")) -> List[Call]:
    """Calls that started in [t0, t1]."""
    return [c for c in list(_RING) if t0 <= c[0] <= t1]


def serial_depth(cs: Iterable[Call]) -> int:
    """The longest chain of calls in which each starts after the previous one ended (greedy by
    end time: the maximum set of pairwise non-overlapping intervals). Zero-length entries
    (file reads) are not round trips and are left out."""
    depth, end = 0, float("-inf")
    for t0, t1, _ in sorted((c for c in cs if c[1] > c[0]), key=lambda c: c[1]):
        if t0 >= end:
            depth += 1
            end = t1
    return depth


def summary(cs: List[Call]) -> Dict[str, object]:
    """Calls by kind and the serial round trips among those the operation waits for
    (background ones are listed apart and not chained)."""
    kinds: Dict[str, int] = {}
    bg: Dict[str, int] = {}
    for _, _, k in cs:
        d = bg if k.endswith(BACKGROUND) else kinds
        k = k[:-len(BACKGROUND)] if k.endswith(BACKGROUND) else k
        d[k] = d.get(k, 0) + 1
    return {"calls": dict(sorted(kinds.items())),
            "serial_round_trips": serial_depth(c for c in cs if not c[2].endswith(BACKGROUND)),
            "background": dict(sorted(bg.items()))}
