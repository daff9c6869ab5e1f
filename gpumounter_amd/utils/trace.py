"""Per-operation span trees with monotonic timings, mirrored to rocprofiler roctx ranges.

The reference has no tracing — only Info log lines per step (e.g. reference:
pkg/server/gpu-mount/server.go:81). Every attach/detach here produces a tree
``attach → {ledger_reserve, placeholder_wait, ledger_read, cgroup_rule, devnodes, verify}``
whose durations are returned to the caller (JSON API), exported as Prometheus histograms, and —
when ``librocprofiler-sdk-roctx`` is present — emitted as roctx push/pop ranges so
``rocprofv3 --marker-trace`` timelines show controller stages next to tenant GPU kernels.
"""
from __future__ import annotations

import contextvars
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

_current: contextvars.ContextVar[Optional["Span"]] = contextvars.ContextVar("gm_span", default=None)

_roctx_lock = threading.Lock()
_roctx = None  # resolved lazily: native host lib or False
_sinks: List[Callable[["Span"], None]] = []


_names: Dict[str, bytes] = {}     # span name → its encoded roctx range name


def _profiled() -> bool:
    """Ranges are emitted when a profiler is attached (rocprofv3 preloads its tool library
    and exports ROCPROF* variables) or when ``GM_ROCTX=on``; ``GM_ROCTX=off`` never. Without a
    profiler the two ctypes calls per span are pure cost on the attach path."""
    mode = os.environ.get("GM_ROCTX", "auto").lower()
    if mode in ("on", "1", "true"):
        return True
    if mode in ("off", "0", "false"):
        return False
    return "rocprofiler" in os.environ.get("LD_PRELOAD", "") or \
        any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def _roctx_lib():
    global _roctx
    if _roctx is None:
        with _roctx_lock:
            if _roctx is None:
                try:
                    from gpumounter_amd import _native

                    lib = _native.host()
                    _roctx = lib if _profiled() and lib.gm_roctx_available() else False
                except Exception:  # noqa: BLE001 - tracing must never break the data path
                    _roctx = False
    return _roctx or None


def set_roctx_enabled(enabled: bool) -> None:
    global _roctx
    with _roctx_lock:
        _roctx = None if enabled else False


def add_sink(fn: Callable[["Span"], None]) -> None:
    """Register a callback invoked with every finished *root* span."""
    _sinks.append(fn)


@dataclass
class Span:
    name: str
    start_ns: int = 0
    end_ns: int = 0
    attrs: Dict[str, object] = field(default_factory=dict)
    children: List["Span"] = field(default_factory=list)
    parent: Optional["Span"] = None
    error: Optional[str] = None

    @property
    def duration_ms(self) -> float:
        end = self.end_ns or time.perf_counter_ns()
        return (end - self.start_ns) / 1e6

    def to_dict(self) -> dict:
        d = {"name": self.name, "ms": round(self.duration_ms, 4)}
        if self.attrs:
            d["attrs"] = dict(self.attrs)
        if self.error:
            d["error"] = self.error
        if self.children:
            d["children"] = [c.to_dict() for c in self.children]
        return d

    def flat(self, prefix: str = "") -> Dict[str, float]:
        """Stage name → total ms (children summed by name)."""
        out: Dict[str, float] = {}
        for c in self.children:
            key = prefix + c.name
            out[key] = out.get(key, 0.0) + c.duration_ms
            for k, v in c.flat(prefix=key + ".").items():
                out[k] = out.get(k, 0.0) + v
        return out


class span:
    """``with span("cgroup_rule", gpu=3): ...`` — nests under the current span (ContextVar)."""

    __slots__ = ("s", "_tok", "_lib", "_rid")

    def __init__(self, name: str, **attrs):
        self.s = Span(name=name, attrs=attrs)

    def __enter__(self) -> Span:
        parent = _current.get()
        self.s.parent = parent
        if parent is not None:
            parent.children.append(self.s)
        self._tok = _current.set(self.s)
        self._lib = _roctx_lib()
        if self._lib is not None:
            # start/stop ranges, not push/pop: spans of concurrent asyncio tasks interleave on
            # one thread, which a per-thread range stack would mis-nest
            name = _names.get(self.s.name)
            if name is None:
                name = _names[self.s.name] = f"gm:{self.s.name}".encode()
            self._rid = self._lib.gm_roctx_start(name)
        self.s.start_ns = time.perf_counter_ns()
        return self.s

    def __exit__(self, et, ev, tb):
        self.s.end_ns = time.perf_counter_ns()
        if ev is not None:
            self.s.error = f"{et.__name__}: {ev}"
        if self._lib is not None:
            self._lib.gm_roctx_stop(self._rid)
        _current.reset(self._tok)
        if self.s.parent is None:
            for fn in list(_sinks):
                try:
                    fn(self.s)
                except Exception:  # noqa: BLE001
                    pass
        return False


def current() -> Optional[Span]:
    return _current.get()


def record(name: str, duration_ns: int, **attrs) -> None:
    """Attach an already-measured stage (e.g. timed inside one native call) as a child of the
    current span, laid out back to back after the previous recorded sibling."""
    parent = _current.get()
    if parent is None or duration_ns <= 0:
        return
    start = parent.children[-1].end_ns if parent.children and parent.children[-1].end_ns \
        else parent.start_ns
    parent.children.append(Span(name=name, start_ns=start, end_ns=start + int(duration_ns),
                                attrs=attrs, parent=parent))


def annotate(**attrs) -> None:
    s = _current.get()
    if s is not None:
        s.attrs.update(attrs)


def mark(name: str) -> None:
    lib = _roctx_lib()
    if lib is not None:
        lib.gm_roctx_mark(name.encode())
