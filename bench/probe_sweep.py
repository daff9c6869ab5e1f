"""Probe-kernel sweep on one MI355X, next to what PyTorch's own kernels reach on the same box.

HBM: copy variants (gm_probe_hbm_copy_variant) and the read-only stream (gm_probe_hbm_read) vs
torch ``dst.copy_(src)`` / ``x.sum()``; MFMA: peak-kernel shapes vs ``torch.matmul`` bf16 (hipBLASLt).
Prints one JSON document. Run on the GPU box: ``python bench/probe_sweep.py``.
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpumounter_amd import _native  # noqa: E402

lib = _native.probe()
lib.gm_probe_hbm_copy_variant.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int,
                                          C.POINTER(C.c_double)]
lib.gm_probe_hbm_read.argtypes = [C.c_int, C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.gm_probe_mfma_peak_variant.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(C.c_double)]
quick = "--quick" in sys.argv
out = {"hbm_copy_GBps": {}, "hbm_read_GBps": {}, "mfma_TFLOPs": {}, "torch": {}}
g = C.c_double(0)
sizes = (1 << 30, 4 << 30)
for variant in ((2, 3, 5, 6) if quick else (0, 1, 2, 3, 4, 5, 6)):
    for bpc in (4, 8):
        for size in sizes:
            rc = lib.gm_probe_hbm_copy_variant(0, variant, size, 10, bpc, C.byref(g))
            out["hbm_copy_GBps"][f"v{variant}_bpc{bpc}_{size >> 30}GiB"] = \
                round(g.value, 1) if rc == 0 else f"err{rc}"
for bpc in (2, 4, 8):
    for size in sizes:
        rc = lib.gm_probe_hbm_read(0, size, 10, bpc, C.byref(g))
        out["hbm_read_GBps"][f"bpc{bpc}_{size >> 30}GiB"] = \
            round(g.value, 1) if rc == 0 else f"err{rc}"
names = {0: "32x32x16x4", 1: "16x16x32x4", 2: "16x16x32x8"}
for shape in ((2,) if quick else (0, 1, 2)):
    for bpc in (4, 8):
        rc = lib.gm_probe_mfma_peak_variant(0, shape, 20000, bpc, C.byref(g))
        out["mfma_TFLOPs"][f"{names[shape]}_bpc{bpc}"] = round(g.value, 1) if rc == 0 else f"err{rc}"

import torch  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


for size in sizes:
    src = torch.ones(size // 4, dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)
    s = timed(lambda: dst.copy_(src), 10)
    out["torch"][f"copy_{size >> 30}GiB_GBps"] = round(2 * size / s / 1e9, 1)
    s = timed(lambda: src.sum(), 10)
    out["torch"][f"sum_{size >> 30}GiB_GBps"] = round(size / s / 1e9, 1)
    del src, dst
for n in (8192,):
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    s = timed(lambda: a @ b, 20)
    out["torch"][f"matmul_bf16_{n}_TFLOPs"] = round(2 * n ** 3 / s / 1e12, 1)
print(json.dumps(out, indent=1))
