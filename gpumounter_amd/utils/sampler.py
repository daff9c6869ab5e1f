"""A statistical CPU profiler for a live daemon: ``setitimer(ITIMER_PROF)`` + the Python stack.

cProfile hooks every call and return, which roughly doubles the cost of the short handlers an
attach runs through and so distorts exactly the split it is meant to measure. This sampler
instead takes the main thread's Python stack every ``interval_s`` of *process CPU time*
(``ITIMER_PROF`` counts every thread, including grpc's C-core threads) and aggregates:

* ``self``: the innermost Python function of each sample;
* ``cum``: every distinct function on the stack (a function's inclusive share);
* ``idle_loop``: samples taken while the event loop thread sat in ``select``/``epoll`` — the
  process was burning CPU in another thread (grpc's poller and completion-queue threads, the
  executor), which this records as such instead of charging it to a Python function.

Config: ``GM_PROFILE_OUT=<path>`` (``{pid}`` replaced) with ``GM_PROFILE_MODE=sample``
(``cprofile``, the default, keeps the deterministic profiler); ``GM_PROFILE_HZ`` (default 2000).
The report is JSON: totals plus the top entries of each table, see :meth:`Sampler.report`.
"""
from __future__ import annotations

import collections
import json
import os
import resource
import signal
import time
from typing import Dict, Optional, Tuple

_Key = Tuple[str, str, int]            # (file, function, first line)
_IDLE = {"select", "poll", "_run_once", "run_forever"}


def _short(path: str) -> str:
    for marker in ("/gpumounter_amd/", "/site-packages/", "/lib/python3"):
        i = path.rfind(marker)
        if i >= 0:
            return path[i + 1:]
    return os.path.basename(path)


def _lib(short: str) -> str:
    """``gpumounter_amd/worker/x.py`` → ``gpumounter_amd/worker``;
    ``lib/python3.10/dist-packages/grpc/aio/_call.py`` → ``grpc``;
    ``lib/python3.10/json/decoder.py`` → ``json``."""
    parts = short.split("/")
    if parts[0] == "gpumounter_amd":
        return "/".join(parts[:2])
    if parts[0] == "lib" and len(parts) > 2:
        rest = parts[2:] if parts[2] not in ("dist-packages", "site-packages") else parts[3:]
        return rest[0] if len(rest) > 1 else rest[0].rsplit(".", 1)[0]
    return parts[0]


class Sampler:
    MAX_DEPTH = 64

    def __init__(self, interval_s: float = 0.0005) -> None:
        self.interval_s = interval_s
        self.samples = 0
        self.idle = 0
        self.self_counts: Dict[_Key, int] = collections.Counter()
        self.cum_counts: Dict[_Key, int] = collections.Counter()
        # innermost gpumounter frame of each non-idle sample: where our own code spends it,
        # whatever library it calls into
        self.own_counts: Dict[_Key, int] = collections.Counter()
        self.lib_counts: Dict[str, int] = collections.Counter()   # leaf's package
        self._prev = None

    def start(self) -> None:
        self._cpu0 = self._cpu()
        self._main0 = time.thread_time()
        self._wall0 = time.monotonic()
        self._prev = signal.signal(signal.SIGPROF, self._on_sample)
        signal.setitimer(signal.ITIMER_PROF, self.interval_s, self.interval_s)

    @staticmethod
    def _cpu() -> float:
        ru = resource.getrusage(resource.RUSAGE_SELF)
        return ru.ru_utime + ru.ru_stime

    def stop(self) -> None:
        signal.setitimer(signal.ITIMER_PROF, 0, 0)
        # the kernel fires ITIMER_PROF at its tick at most (250-1000 Hz), whatever was asked:
        # the CPU totals come from getrusage, the samples only give the shares
        self.cpu_s = self._cpu() - self._cpu0
        self.main_cpu_s = time.thread_time() - self._main0
        self.wall_s = time.monotonic() - self._wall0
        if self._prev is not None:
            signal.signal(signal.SIGPROF, self._prev)
            self._prev = None

    @staticmethod
    def _key(f) -> _Key:
        c = f.f_code
        return (_short(c.co_filename), c.co_name, c.co_firstlineno)

    def _on_sample(self, signum, frame) -> None:
        if frame is None:
            return
        self.samples += 1
        leaf = self._key(frame)
        # the loop thread blocked in select(): the CPU went to another thread
        if leaf[1] in _IDLE and leaf[0].endswith(("selectors.py", "base_events.py")):
            self.idle += 1
            return
        self.self_counts[leaf] += 1
        self.lib_counts[_lib(leaf[0])] += 1
        seen = set()
        own = None
        f, depth = frame, 0
        while f is not None and depth < self.MAX_DEPTH:
            k = self._key(f)
            if k not in seen:
                seen.add(k)
                self.cum_counts[k] += 1
            if own is None and k[0].startswith("gpumounter_amd/"):
                own = k
            f = f.f_back
            depth += 1
        if own is not None:
            self.own_counts[own] += 1

    def report(self, top: int = 40) -> dict:
        n = max(self.samples, 1)

        def table(c):
            return [{"fn": k if isinstance(k, str) else f"{k[0]}:{k[2]} {k[1]}",
                     "samples": v, "pct": round(100.0 * v / n, 2)}
                    for k, v in c.most_common(top)]
        return {"interval_s": self.interval_s, "samples": self.samples,
                "cpu_s": round(getattr(self, "cpu_s", 0.0), 3),
                "main_thread_cpu_s": round(getattr(self, "main_cpu_s", 0.0), 3),
                "wall_s": round(getattr(self, "wall_s", 0.0), 3),
                "idle_loop_samples": self.idle,
                "idle_loop_pct": round(100.0 * self.idle / n, 2),
                "lib": table(self.lib_counts), "self": table(self.self_counts),
                "cum": table(self.cum_counts), "own": table(self.own_counts)}

    def dump(self, path: str, extra: Optional[dict] = None) -> None:
        rep = self.report()
        if extra:
            rep.update(extra)
        with open(path, "w") as fh:
            json.dump(rep, fh, indent=1)
