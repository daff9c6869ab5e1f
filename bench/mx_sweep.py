"""MX-MFMA peak forms on one MI355X: 16x16x128 × 8 chains vs 32x32x64 × 4 / × 8, at several
workgroups per CU, fp8 and fp4; best of three runs each.

    python bench/mx_sweep.py > mx_sweep.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpumounter_amd.ops import mx  # noqa: E402


def main():
    out = []
    for fmt in ("fp8", "fp4"):
        for variant in (0, 1, 2):
            for bpc in (2, 4, 8):
                it = 20000 if variant == 0 else 10000
                t = max(mx.peak(0, fmt, it, bpc, variant)[0] for _ in range(3))
                out.append({"fmt": fmt, "variant": variant, "blocks_per_cu": bpc,
                            "tflops": round(t, 1)})
                print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
