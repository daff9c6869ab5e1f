"""Process-level latency tuning for the daemons.

After startup almost every Python object (modules, protobuf descriptors, gRPC/aiohttp machinery,
informer caches) lives for the whole process, yet a full (generation-2) collection walks all of
them: measured 30+ ms pauses on the attach path on a busy host. ``gc.freeze()`` moves what exists
after startup into the permanent generation, so later full collections only walk what requests
allocate. The young-generation threshold stays small: raising it (tried 50 000) trades many
sub-ms pauses for rare 25-40 ms ones, which is worse for the p99.
"""
from __future__ import annotations

import gc
import json
import os


def parse_cpus(spec: str) -> set:
    """``"2-3,8"`` → {2, 3, 8} (the cpuset list format)."""
    out = set()
    for part in filter(None, (p.strip() for p in spec.split(","))):
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def pin_cpus(spec: str) -> set:
    """Pin this process (and the threads it starts afterwards: grpc's, the executor's) to the
    CPUs of ``spec`` (config ``cpu_affinity``), as a static-CPU-manager node gives a Guaranteed
    pod exclusive cores: no other process runs there, so a request's wake-ups find a warm,
    idle core. CPUs this process may not use are dropped; none left → unchanged. Returns the
    set now in force."""
    want = parse_cpus(spec)
    if not want or not hasattr(os, "sched_setaffinity"):
        return set(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else set()
    allowed = os.sched_getaffinity(0)
    use = want & allowed
    if use:
        os.sched_setaffinity(0, use)
    return set(os.sched_getaffinity(0))


def tune_gc(freeze: bool = True) -> None:
    if freeze:
        gc.collect()
        gc.freeze()


_gc_t0 = [0.0]
_gc_watching = [False]
gc_pauses: list = []          # (generation, ms) of collections over the threshold


def watch_gc_pauses(threshold_ms: float = 5.0, logger=None) -> None:
    """Log every garbage collection that stops the process for more than ``threshold_ms``
    (generation, pause, objects collected): tail-latency attribution for the daemons."""
    import time

    def cb(phase: str, info: dict) -> None:
        if phase == "start":
            _gc_t0[0] = time.perf_counter()
            return
        ms = (time.perf_counter() - _gc_t0[0]) * 1e3
        if ms >= threshold_ms:
            gc_pauses.append((info.get("generation"), round(ms, 2)))
            del gc_pauses[:-100]
            if logger is not None:
                logger.warning("gc pause: generation %s, %.1f ms, %s collected",
                               info.get("generation"), ms, info.get("collected"))

    if not _gc_watching[0]:
        _gc_watching[0] = True
        gc.callbacks.append(cb)


def write_ready_file(path: str, info: dict) -> None:
    """Atomically publish what a daemon bound (config ``ready_file``)."""
    if not path:
        return
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as fh:
        json.dump(info, fh)
    os.replace(tmp, path)
