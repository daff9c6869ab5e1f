"""BPF_PROG_LOAD (verifier + JIT) cost of the cgroup-device programs, in isolation (root).

Straight-line programs (one block per device, gm_bpf_dev_build) grow with the device count; the
set-mode program (gm_bpf_dev_build_set) is one map lookup whatever the count. Median of 50
loads each; prints one JSON line.
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
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
