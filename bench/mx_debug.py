"""Localize an MX-MFMA numerics mismatch: random data in A only, B only, both, scales only, all.

    python bench/mx_debug.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpumounter_amd.ops import mx  # noqa: E402


def case(a, b, sa, sb):
    sa_l = np.array([sa[ln & 15, ln >> 4] for ln in range(64)], np.uint8)
    sb_l = np.array([sb[ln & 15, ln >> 4] for ln in range(64)], np.uint8)
    got = mx.c_from_lanes(mx.tile(0, mx.a_lanes(a), mx.b_lanes(b), sa_l, sb_l)).astype(np.float64)
    want = mx.reference(a, b, sa, sb)
    return {"err": float(np.max(np.abs(got - want))), "scale": float(np.max(np.abs(want))),
            "got00": float(got[0, 0]), "want00": float(want[0, 0])}


def main():
    rng = np.random.default_rng(0)
    one = mx.e4m3_encode(1.0)
    pos = np.array([c for c in range(1, 0x7F) if mx.e4m3_decode(np.uint8(c)) <= 8], np.uint8)
    allf = np.array([c for c in range(256) if (c & 0x7F) != 0x7F and
                     abs(mx.e4m3_decode(np.uint8(c))) <= 8], np.uint8)
    normal_pos = np.array([c for c in pos if (c >> 3) & 0xF], np.uint8)
    ones_a = np.full((16, 128), one, np.uint8)
    ones_b = np.full((128, 16), one, np.uint8)
    s1 = np.full((16, 4), 127, np.uint8)
    rs = lambda: rng.integers(123, 132, size=(16, 4)).astype(np.uint8)  # noqa: E731
    out = {
        "randA_pos": case(rng.choice(pos, (16, 128)), ones_b, s1, s1),
        "randA_normal_pos": case(rng.choice(normal_pos, (16, 128)), ones_b, s1, s1),
        "randA_signed": case(rng.choice(allf, (16, 128)), ones_b, s1, s1),
        "randB_pos": case(ones_a, rng.choice(pos, (128, 16)), s1, s1),
        "randAB_pos": case(rng.choice(pos, (16, 128)), rng.choice(pos, (128, 16)), s1, s1),
        "scalesA": case(ones_a, ones_b, rs(), s1),
        "scalesB": case(ones_a, ones_b, s1, rs()),
        "scalesAB": case(ones_a, ones_b, rs(), rs()),
        "all": case(rng.choice(allf, (16, 128)), rng.choice(allf, (128, 16)), rs(), rs()),
    }
    # one-hot value sweep: A[0][0] = code, everything else 0, B = ones → C[0][*] = value
    zeros_a = np.zeros((16, 128), np.uint8)
    bad = []
    for code in range(256):
        if (code & 0x7F) == 0x7F:
            continue
        a = zeros_a.copy()
        a[0, 0] = code
        r = case(a, ones_b, s1, s1)
        if r["got00"] != r["want00"]:
            bad.append((code, r["got00"], r["want00"]))
    out["onehot_value_mismatches"] = bad[:40]
    out["onehot_value_mismatch_count"] = len(bad)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
