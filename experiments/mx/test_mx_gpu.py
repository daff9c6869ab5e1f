"""The MX probes on a real MI355X (not part of the driver's GPU gate: run by hand,
``python -m pytest experiments/mx -q``)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

# a real KFD with GPU nodes (a bare /dev/kfd node without the driver behind it is not one: bench.py
# uses the same probe), and the gpu marker so a CPU run (-m "not gpu") never collects them
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.isdir("/sys/class/kfd/kfd/topology/nodes"),
                                 reason="needs an MI355X")]


# ------------------------------------------------------------------ block-scaled (MX) MFMA
def test_mx_fp8_tile_matches_host_reference():
    """One v_mfma_scale_f32_16x16x128_f8f6f4 on random OCP e4m3 data with random per-block E8M0
    scales against the float64 host reference (gpumounter_amd/ops/mx.py)."""
    import mx

    for seed in range(3):
        r = mx.check_fp8(0, seed)
        assert r["ok"], r


def test_mx_pipes_reach_their_rate_and_are_deterministic():
    import mx

    for fmt, floor in (("fp8", 3000.0), ("fp4", 5000.0)):
        t1, s1 = mx.peak(0, fmt, 2000)
        t2, s2 = mx.peak(0, fmt, 2000)
        assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32)), fmt
        assert np.all(np.isfinite(s1)) and max(t1, t2) > floor, (fmt, t1, t2)


def test_mx_burn_in_reports_no_mismatch():
    import mx

    r = mx.burn_in(0, 1.0, "fp8")
    assert r["ok"] and r["launches"] >= 2, r
