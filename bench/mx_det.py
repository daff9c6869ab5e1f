"""Run-to-run bit equality of the MX-MFMA peak kernel's per-wave sums across iteration counts and
occupancy, plus the fp8 tile numerics check with the measured lane map.

    python bench/mx_det.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpumounter_amd.ops import mx  # noqa: E402


def main():
    out = {"check_fp8": [mx.check_fp8(0, s) for s in range(4)]}
    for fmt in ("fp8", "fp4"):
        for it, bpc in ((20000, 1), (20000, 8), (2000, 8), (200, 8), (20, 8)):
            runs = [mx.peak(0, fmt, it, bpc) for _ in range(3)]
            u = [r[1].view(np.uint32) for r in runs]
            diff = [int(np.sum(u[0] != x)) for x in u[1:]]
            rel = max(float(np.max(np.abs(runs[0][1] - r[1]) / np.maximum(np.abs(runs[0][1]), 1e-30)))
                      for r in runs[1:])
            where = np.nonzero(u[0] != u[1])[0][:8].tolist()
            out[f"{fmt}_{it}_{bpc}"] = {"tflops": [round(r[0], 1) for r in runs],
                                       "waves": len(u[0]), "differing": diff,
                                       "max_rel": rel, "first_differing_waves": where}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
