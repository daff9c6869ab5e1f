"""Which elements each lane's E8M0 scale covers in v_mfma_scale_f32_16x16x128_f8f6f4 (fp8), and
whether repeated MX-MFMAs on the same data agree bit for bit.

A = B = 1.0 everywhere and every scale 2^0 gives C = 128. Raising one lane's A (or B) scale to
2^1 adds 1 to C[r][c] for every element of row r (col c) that the scale covers.

    python bench/mx_scale.py > mx_scale.json
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpumounter_amd.ops import mx  # noqa: E402


def run(sa, sb, a=None, b=None):
    one = mx.e4m3_encode(1.0)
    a = np.full((64, 32), one, np.uint8) if a is None else a
    b = np.full((64, 32), one, np.uint8) if b is None else b
    return mx.c_from_lanes(mx.tile(0, a, b, sa, sb)).astype(np.float64)


def main():
    base = np.full(64, 127, np.uint8)
    out = {"uniform": float(run(base, base)[0, 0])}
    for name in ("a", "b"):
        per_lane = {}
        for lane in range(64):
            s = base.copy()
            s[lane] = 128
            d = run(s, base) if name == "a" else run(base, s)
            delta = d - 128.0
            nz = np.argwhere(delta != 0)
            per_lane[lane] = {"cells": len(nz),
                              "rows": sorted({int(r) for r, _ in nz}),
                              "cols": sorted({int(c) for _, c in nz}),
                              "delta": sorted({float(delta[r, c]) for r, c in nz})}
        out[name] = {str(k): v for k, v in per_lane.items() if k in (0, 1, 15, 16, 17, 31, 32, 48, 63)}
        out[name + "_summary"] = sorted({(len(v["rows"]), len(v["cols"]), tuple(v["delta"]))
                                         for v in per_lane.values()})
    # determinism: the same random tile ten times
    rng = np.random.default_rng(1)
    finite = np.array([c for c in range(256) if (c & 0x7F) != 0x7F], np.uint8)
    a = rng.choice(finite, size=(64, 32)).astype(np.uint8)
    b = rng.choice(finite, size=(64, 32)).astype(np.uint8)
    sa = rng.integers(120, 134, size=64).astype(np.uint8)
    sb = rng.integers(120, 134, size=64).astype(np.uint8)
    runs = [mx.tile(0, a, b, sa, sb) for _ in range(10)]
    out["tile_bitwise_equal"] = all(np.array_equal(runs[0].view(np.uint32), r.view(np.uint32))
                                    for r in runs)
    # the peak kernel's sums across launches, a few iteration counts
    det = {}
    for it in (1, 2, 16, 1000):
        sums = [mx.peak(0, "fp8", it, 1)[1] for _ in range(3)]
        det[it] = {"equal": all(np.array_equal(sums[0].view(np.uint32), s.view(np.uint32))
                                for s in sums),
                   "differing_waves": int(np.sum(sums[0].view(np.uint32) != sums[1].view(np.uint32))),
                   "first": [float(x) for x in sums[0][:4]], "second": [float(x) for x in sums[1][:4]]}
    out["peak_determinism"] = det
    print(json.dumps(out, default=str))


if __name__ == "__main__":
    main()
