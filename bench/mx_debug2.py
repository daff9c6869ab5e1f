"""Which lane's E8M0 scale multiplies each A / B register element of the fp8 MX-MFMA.

A one-hot 1.0 at (lane L, byte J), B all ones, every lane's A scale distinct (2^(l-40)): the output
row's value names the scale's lane. Same for B with A all ones.

    python bench/mx_debug2.py

Measured on MI355X (profiles/r3_mx/scale_lanes.json): byte j of lane l is scaled by lane
(l & 15) + 16 s with s = (l >> 5) for j < 16 and s = 2 + (l >> 5) for j ≥ 16, i.e. k = 16 (l >> 4)
+ j, or 64 + 16 (l >> 4) + (j - 16); "own_lane_scale" is therefore false.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpumounter_amd.ops import mx  # noqa: E402


def main():
    one = mx.e4m3_encode(1.0)
    ones = np.full((64, 32), one, np.uint8)
    distinct = (np.arange(64) + 87).astype(np.uint8)      # 2^(l-40)
    s1 = np.full(64, 127, np.uint8)
    res = {"a": {}, "b": {}}
    for side in ("a", "b"):
        for lane in range(64):
            for j in (0, 31):
                x = np.zeros((64, 32), np.uint8)
                x[lane, j] = one
                if side == "a":
                    c = mx.c_from_lanes(mx.tile(0, x, ones, distinct, s1))
                    vals = c[np.any(c != 0, axis=1)]
                else:
                    c = mx.c_from_lanes(mx.tile(0, ones, x, s1, distinct))
                    vals = c[:, np.any(c != 0, axis=0)].T
                v = sorted({float(t) for t in np.ravel(vals)})
                lanes = [int(round(np.log2(t))) + 40 for t in v if t > 0]
                res[side][f"{lane},{j}"] = lanes
    same = {s: all(v == [int(k.split(",")[0])] for k, v in res[s].items()) for s in res}
    print(json.dumps({"own_lane_scale": same,
                      "a_sample": {k: v for k, v in list(res["a"].items())[::9]},
                      "b_sample": {k: v for k, v in list(res["b"].items())[::9]}}))


if __name__ == "__main__":
    main()
