#!/usr/bin/env python3
"""The device guard's cost on the worker's event loop, per tick, with N hot containers.

    python bench/guard_bench.py [--containers 64] [--passes 300] [--backend real|emulated|v1]

Every ``device_guard_period_s`` (1 s) the worker fingerprints the device control of each hot
container (worker/reconciler.py): cgroup v2 one ``BPF_PROG_QUERY`` (+ program info), cgroup v1
one ``devices.list`` read. Round 4 did that synchronously on the loop that also serves AddGPU;
now the kernel reads run in a thread and the loop keeps only the bookkeeping and the compare.
This prints, per pass: ``sync_ms`` (the round-4 pass, all on the loop) and ``on_loop_ms`` /
``wall_ms`` of the threaded pass, p50 and max, as one JSON line.

``--backend real`` (root: a private cgroup2 mount with a runc-style program attached to every
container cgroup and gpumounter's program installed by the production V2BpfBackend);
``emulated`` (the recording backend's state file per cgroup); ``v1`` (devices.allow/deny files).
"""
import argparse
import asyncio
import json
import os
import shutil
import statistics
import sys
import tempfile
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpumounter_amd.models.device import DeviceNode  # noqa: E402
from gpumounter_amd.node import cgroup  # noqa: E402
from gpumounter_amd.worker.reconciler import Reconciler  # noqa: E402


def _setup(backend: str, n: int):
    """(backend object, [cgroup dirs], cleanup)"""
    grant = [DeviceNode("/dev/dri/renderD128", 226, 128), DeviceNode("/dev/kfd", 511, 0)]
    if backend == "real":
        from gpumounter_amd.fakes.realnode import RealNodeSandbox, attach_runtime_program
        sb = RealNodeSandbox().__enter__()
        be = cgroup.V2BpfBackend(sb.bpffs, True)
        dirs = []
        for i in range(n):
            d = os.path.join(sb.cgroup_root, f"ctr{i}")
            os.makedirs(d, exist_ok=True)
            attach_runtime_program(d)
            be.apply(d, grant, [], grant)
            dirs.append(d)
        return be, dirs, lambda: sb.__exit__(None, None, None)
    root = tempfile.mkdtemp(prefix="gm-guard-", dir="/dev/shm" if os.access("/dev/shm", os.W_OK)
                            else None)
    dirs = []
    for i in range(n):
        d = os.path.join(root, f"ctr{i}")
        os.makedirs(d)
        dirs.append(d)
    if backend == "v1":
        be = cgroup.V1Backend()
        for d in dirs:
            open(os.path.join(d, cgroup.FAKE_MARKER), "w").close()
            for f in ("devices.allow", "devices.deny"):
                open(os.path.join(d, f), "w").close()
    else:
        be = cgroup.V2RecordingBackend()
    for d in dirs:
        be.apply(d, grant, [], grant)
    return be, dirs, lambda: shutil.rmtree(root, ignore_errors=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--containers", type=int, default=64)
    ap.add_argument("--passes", type=int, default=300)
    ap.add_argument("--backend", choices=("real", "emulated", "v1"), default="emulated")
    args = ap.parse_args()
    be, dirs, cleanup = _setup(args.backend, args.containers)
    try:
        entries = [SimpleNamespace(rules=["c 226:128 rw"], cgdir=d, namespace="default",
                                   pod=f"t{i}") for i, d in enumerate(dirs)]
        hm = SimpleNamespace(journal=SimpleNamespace(entries=lambda: entries), expected={},
                             backend=be)
        svc = SimpleNamespace(hm=hm, cfg=SimpleNamespace(device_guard_period_s=1.0))
        rec = Reconciler.__new__(Reconciler)      # only the guard's state is needed
        rec.svc, rec.guard_repairs, rec._stopping = svc, 0, False   # noqa: SLF001
        rec._kick = lambda key: None                                 # noqa: SLF001

        async def run():
            rec.guard_once()                      # baseline (first sight)
            sync, on_loop, wall = [], [], []
            for _ in range(args.passes):
                t0 = time.perf_counter()
                rec.guard_once()
                sync.append((time.perf_counter() - t0) * 1e3)
            fp = be.fingerprint
            for _ in range(args.passes):
                # guard_pass, with its two loop-side segments timed apart from the thread
                t0 = time.perf_counter()
                targets = rec._guard_targets()                         # noqa: SLF001
                before = dict(hm.expected)
                t1 = time.perf_counter()
                seen = await asyncio.to_thread(rec._fingerprints, fp,  # noqa: SLF001
                                               [d for _, d in targets])
                t2 = time.perf_counter()
                kicked = rec._guard_compare(targets, seen, before)     # noqa: SLF001
                t3 = time.perf_counter()
                assert not kicked
                on_loop.append(((t1 - t0) + (t3 - t2)) * 1e3)
                wall.append((t3 - t0) * 1e3)
            return sync, on_loop, wall
        sync, on_loop, wall = asyncio.run(run())

        def st(xs):
            return {"p50": round(statistics.median(xs), 4), "max": round(max(xs), 4)}
        print(json.dumps({"backend": args.backend, "containers": args.containers,
                          "passes": args.passes, "sync_ms": st(sync),
                          "on_loop_ms": st(on_loop), "wall_ms": st(wall)}))
    finally:
        cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
