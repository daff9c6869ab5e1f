"""BPF_PROG_LOAD (verifier + JIT) cost of the cgroup-device programs, in isolation (root).

Straight-line programs (one block per device, gm_bpf_dev_build) grow with the device count; the
set-mode program (gm_bpf_dev_build_set) is one map lookup whatever the count. Median of 50
loads each, then whole install/verify/restore cycles of the backend on a real cgroup2
hierarchy in both modes (install_cycles); prints one JSON line.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpumounter_amd import _native  # noqa: E402

_SYS_BPF = 321  # x86_64


def _map(libc, mtype: int, key: int, value: int, entries: int) -> int:
    attr = (C.c_uint32 * 32)(mtype, key, value, entries)
    fd = libc.syscall(_SYS_BPF, 0, attr, 128)       # BPF_MAP_CREATE
    if fd < 0:
        raise OSError(C.get_errno(), "BPF_MAP_CREATE")
    return fd


def _median_load_ms(lib, words, n: int, reps: int = 50) -> float:
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fd = lib.gm_bpf_dev_load(words, n, b"gm_devallow", None, 0)
        ts.append(time.perf_counter() - t0)
        if fd < 0:
            raise OSError(-fd, "BPF_PROG_LOAD")
        os.close(fd)
    return round(statistics.median(ts) * 1e3, 4)


def main() -> int:
    lib = _native.host()
    libc = C.CDLL(None, use_errno=True)
    chain = _map(libc, 3, 4, 4, 1)                   # PROG_ARRAY (tail-call slot)
    setm = _map(libc, 1, 12, 4, 512)                 # HASH allow set
    out = {"straight_line": {}, "set_mode": {}}
    for gpus in (1, 2, 4, 8):
        nodes = 1 + 2 * gpus                         # /dev/kfd + renderD + card per GPU
        rules = (_native.DevRule * nodes)(*[_native.DevRule(b"c", 6, 1, 0, 226, 128 + i)
                                            for i in range(nodes)])
        need = -lib.gm_bpf_dev_build(rules, nodes, 0, chain, None, 0)
        buf = (C.c_uint64 * need)()
        k = lib.gm_bpf_dev_build(rules, nodes, 0, chain, buf, need)
        out["straight_line"][gpus] = {"insns": k, "load_ms": _median_load_ms(lib, buf, k)}
    need = -lib.gm_bpf_dev_build_set(setm, None, 0, 0, chain, None, 0)
    buf = (C.c_uint64 * need)()
    k = lib.gm_bpf_dev_build_set(setm, None, 0, 0, chain, buf, need)
    out["set_mode"] = {"insns": k, "load_ms": _median_load_ms(lib, buf, k)}
    os.close(chain)
    os.close(setm)
    out["install_cycle"] = install_cycles(lib)
    print(json.dumps(out))
    return 0


def install_cycles(lib, reps: int = 40) -> dict:
    """The backend on a real cgroup2 hierarchy with a runc-style program attached: attach N
    GPUs to a Pod that has none (wrap), read the grants back (the attach verify), detach them
    all (restore); and growing a Pod 1 → 8 one GPU at a time. Medians in ms, both modes."""
    import subprocess
    import tempfile
    import uuid

    from gpumounter_amd.fakes.realnode import attach_runtime_program
    from gpumounter_amd.models.device import DeviceNode
    from gpumounter_amd.node.cgroup import V2BpfBackend

    mnt = tempfile.mkdtemp(prefix="gm-bpfload-cg2-")
    pins = tempfile.mkdtemp(prefix="gm-bpfload-pins-")
    subprocess.run(["mount", "-t", "cgroup2", "none", mnt], check=True)
    subprocess.run(["mount", "-t", "bpf", "bpf", pins], check=True)
    cg = os.path.join(mnt, "gm-bpfload-" + uuid.uuid4().hex[:8])
    os.mkdir(cg)
    res = {}
    try:
        attach_runtime_program(cg)
        gpu = [[DeviceNode(f"/dev/dri/renderD{128 + i}", 226, 128 + i),
                DeviceNode(f"/dev/dri/card{i}", 226, i)] for i in range(8)]
        kfd = DeviceNode("/dev/kfd", 511, 0)
        for mode, straight in (("straight_line", 1), ("set_mode", 0)):
            be = V2BpfBackend(pins, set_mode=not straight)
            r = {}
            for n in (1, 8):
                want = [kfd] + [x for g in gpu[:n] for x in g]
                att, ver, det = [], [], []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    be.apply(cg, want, [], want)
                    t1 = time.perf_counter()
                    got = be.allowed(cg)
                    t2 = time.perf_counter()
                    be.apply(cg, [], want, [])
                    t3 = time.perf_counter()
                    assert {(x.major, x.minor) for x in want} <= got
                    att.append(t1 - t0)
                    ver.append(t2 - t1)
                    det.append(t3 - t2)
                r[f"attach_{n}gpu_ms"] = round(statistics.median(att) * 1e3, 4)
                r[f"verify_{n}gpu_ms"] = round(statistics.median(ver) * 1e3, 4)
                r[f"detach_all_{n}gpu_ms"] = round(statistics.median(det) * 1e3, 4)
            grow = []
            for _ in range(reps // 4):
                have = [kfd]
                for i in range(8):
                    t0 = time.perf_counter()
                    be.apply(cg, gpu[i], [], have + gpu[i])
                    grow.append(time.perf_counter() - t0)
                    have = have + gpu[i]
                be.apply(cg, [], have, [])
            r["grow_step_ms"] = round(statistics.median(grow) * 1e3, 4)
            res[mode] = r
    finally:
        lib.gm_bpf_dev_straight_line(0)
        try:
            os.rmdir(cg)
        except OSError:
            pass
        subprocess.run(["umount", pins], check=False)
        subprocess.run(["umount", mnt], check=False)
        os.rmdir(pins)
        os.rmdir(mnt)
    return res


if __name__ == "__main__":
    sys.exit(main())
