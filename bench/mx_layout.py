"""Discover the lane map of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3) on the GPU with exact data.

For every A register byte (lane L, byte J) one MFMA runs with A one-hot there (1.0) and every B
byte holding a distinct e4m3 code of its own (lane half, byte) index. The nonzero output row
names the A element's row; the value in column c names which B byte of that column shares its
K index. The C/D map (col = lane & 15, row = 4 (lane >> 4) + reg) is the documented gfx950 one.
Prints a summary and whether the simple hypothesis holds:
  A: lane l holds row l & 15, k = 32 (l >> 4) + byte;   B: lane l holds col l & 15, same k.
It does for rows and for the A↔B pairing, which is all unit scales can see. Which 32-wide block
each byte belongs to (what a scale multiplies) is bench/mx_debug2.py's question: bytes 0-15 and
16-31 of a lane sit 64 apart in k (gpumounter_amd/ops/mx.py k_index).

    python bench/mx_layout.py > mx_layout.json
"""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from gpumounter_amd import _native  # noqa: E402
from gpumounter_amd.ops import mx  # noqa: E402


def tile(a, b, sa, sb):
    c = np.zeros((64, 4), np.float32)
    rc = _native.probe().gm_probe_mx_tile(0, 0, a.ctypes.data, b.ctypes.data, sa.ctypes.data,
                                           sb.ctypes.data, c.ctypes.data)
    if rc:
        raise RuntimeError(f"mx_tile rc={rc}")
    return c


def main():
    one = mx.e4m3_encode(1.0)
    # B byte (lane l, byte j) = code of idx = (l >> 4) * 32 + j, signed to get 128 distinct values
    b = np.zeros((64, 32), np.uint8)
    val_to_idx = {}
    for lane in range(64):
        for j in range(32):
            idx = (lane >> 4) * 32 + j
            code = idx + 1 if idx < 126 else 0x80 | (idx - 125)
            b[lane, j] = code
            val_to_idx[float(mx.e4m3_decode(np.uint8(code)))] = idx
    s127 = np.full(64, 127, np.uint8)
    amap = {}
    bad = 0
    for lane in range(64):
        for j in range(32):
            a = np.zeros((64, 32), np.uint8)
            a[lane, j] = one
            c = tile(a, b, s127, s127)
            out = mx.c_from_lanes(c)          # [16 rows][16 cols]
            rows = [r for r in range(16) if np.any(out[r] != 0)]
            if len(rows) != 1:
                bad += 1
                continue
            r = rows[0]
            idxs = [val_to_idx.get(float(out[r, col]), -1) for col in range(16)]
            amap[(lane, j)] = (r, idxs[0] if len(set(idxs)) == 1 else idxs)
    simple = all(v == ((lane & 15), (lane >> 4) * 32 + j) for (lane, j), v in amap.items())
    print(json.dumps({"mapped": len(amap), "unmapped": bad, "simple_hypothesis": simple,
                      "sample": {f"{k[0]},{k[1]}": v for k, v in list(amap.items())[:40:3]}}))


if __name__ == "__main__":
    main()
