import ctypes as C, json, sys
sys.path.insert(0, "/root/repo")
from gpumounter_amd import _native
lib = _native.probe()
lib.gm_probe_hbm_copy_variant.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_double)]
lib.gm_probe_mfma_peak_variant.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
out = {"hbm": {}, "mfma": {}}
g = C.c_double(0)
for variant in (0, 1, 2, 3, 4):
    for bpc in (2, 4, 8):
        for size in (1 << 30, 4 << 30):
            rc = lib.gm_probe_hbm_copy_variant(0, variant, size, 10, bpc, C.byref(g))
            out["hbm"][f"v{variant}_bpc{bpc}_{size >> 30}GiB"] = round(g.value, 1) if rc == 0 else f"err{rc}"
names = {0: "32x32x16x4", 1: "16x16x32x4", 2: "16x16x32x8"}
for shape in (0, 1, 2):
    for bpc in (1, 2, 4, 8):
        rc = lib.gm_probe_mfma_peak_variant(0, shape, 20000, bpc, C.byref(g))
        out["mfma"][f"{names[shape]}_bpc{bpc}"] = round(g.value, 1) if rc == 0 else f"err{rc}"
print(json.dumps(out, indent=1))
