"""Probe kernels as a short fixed workload for rocprofv3 PMC passes (profiles/history/r1_pmc_probe).

    rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d DIR -- python3 bench/pmc_probe.py

Dispatches: 3 × read stream over 1 GiB, 3 × copy of 1 GiB, 2 × MFMA bf16 peak (16x16x32 × 8
chains, 8 blocks/CU). Byte and FLOP totals per dispatch are printed as JSON, for turning the
counters into achieved HBM bytes and MFMA utilisation.
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
lib.gm_probe_mfma_peak_variant.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(C.c_double)]
g = C.c_double(0)
out = {}
assert lib.gm_probe_hbm_read(0, 1 << 30, 3, 2, C.byref(g)) == 0
out["read_GBps"] = round(g.value, 1)
assert lib.gm_probe_hbm_copy_variant(0, 2, 1 << 30, 3, 8, C.byref(g)) == 0
out["copy_GBps"] = round(g.value, 1)
assert lib.gm_probe_mfma_peak_variant(0, 2, 20000, 8, C.byref(g)) == 0
out["mfma_TFLOPs"] = round(g.value, 1)
out["bytes"] = {"read_dispatch": 1 << 30, "copy_dispatch_read": 1 << 30,
                "copy_dispatch_write": 1 << 30}
out["mfma_dispatch_flops"] = 2 * 16 * 16 * 32 * 8 * 20000 * 256 * 8 * 4
print(json.dumps(out))
