"""Host side of the block-scaled (MX) MFMA check (experiments/mx/mx.py): the OCP e4m3
decoder, the measured lane map and the reference. The tile runs here on a CPU emulation of the
map measured on MI355X (round-3 probe scripts, removed; results in profiles/r3_mx/); tests/test_gpu.py runs it on
the matrix core."""
import numpy as np
import pytest

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mx  # noqa: E402


def emulate(af, bf, sa, sb, k_of=mx.k_index):
    """The fp8 MX-MFMA as measured: lane l holds row/col l & 15 at k = k_of(l, byte); the scale of
    row/col r, block s comes from lane r + 16 s; C/D col = l & 15, row = 4 (l >> 4) + reg."""
    A, B = np.zeros((16, 128)), np.zeros((128, 16))
    SA, SB = np.zeros((16, 4)), np.zeros((16, 4))
    for ln in range(64):
        for j in range(32):
            k = k_of(ln, j)
            A[ln & 15, k] = mx.e4m3_decode(af[ln, j])
            B[k, ln & 15] = mx.e4m3_decode(bf[ln, j])
        SA[ln & 15, ln >> 4], SB[ln & 15, ln >> 4] = sa[ln], sb[ln]
    C = (A * np.repeat(mx.e8m0(SA), 32, axis=1)) @ (B * np.repeat(mx.e8m0(SB), 32, axis=1).T)
    out = np.zeros((64, 4), np.float32)
    for ln in range(64):
        for q in range(4):
            out[ln, q] = C[4 * (ln >> 4) + q, ln & 15]
    return out


def test_e4m3_is_the_ocp_format():
    d = mx.e4m3_decode(np.arange(256, dtype=np.uint8))
    assert d[0x38] == 1.0 and d[0x7E] == 448.0 and d[0xFE] == -448.0   # OCP max, not FNUZ's 240
    assert d[0x01] == 2.0 ** -9 and d[0x08] == 2.0 ** -6                # subnormal, min normal
    assert np.isnan(d[0x7F]) and np.isnan(d[0xFF]) and d[0x80] == 0.0   # no FNUZ NaN at 0x80
    assert np.sum(np.isfinite(d) & (d > 0)) == 126
    assert mx.e4m3_encode(-0.5) == 0xB0
    with pytest.raises(ValueError):
        mx.e4m3_encode(0.3)


def test_lane_map_covers_every_k_once_per_row():
    for row in range(16):
        ks = sorted(mx.k_index(ln, j) for ln in range(row, 64, 16) for j in range(32))
        assert ks == list(range(128))
    # a lane spans two scale blocks: bytes 0-15 and 16-31 sit 64 apart in k
    assert mx.k_index(0, 15) == 15 and mx.k_index(0, 16) == 64 and mx.k_index(48, 31) == 127


def test_check_passes_on_the_measured_map_and_rejects_the_naive_one(monkeypatch):
    monkeypatch.setattr(mx, "tile", lambda dev, af, bf, sa, sb, fmt="fp8": emulate(af, bf, sa, sb))
    for seed in range(3):
        r = mx.check_fp8(0, seed)
        assert r["ok"] and r["max_err_over_abs_sum"] < 1e-6, r
    # the map a first guess gives (k = 32 (l >> 4) + byte): right with unit scales, wrong here
    naive = lambda ln, j: 32 * (ln >> 4) + j  # noqa: E731
    monkeypatch.setattr(mx, "tile", lambda dev, af, bf, sa, sb, fmt="fp8":
                        emulate(af, bf, sa, sb, k_of=naive))
    assert not mx.check_fp8(0, 0)["ok"]


def test_reference_applies_block_scales():
    one = mx.e4m3_encode(1.0)
    a = np.full((16, 128), one, np.uint8)
    b = np.full((128, 16), one, np.uint8)
    sa = np.full((16, 4), 127, np.uint8)
    sb = np.full((16, 4), 127, np.uint8)
    sa[3, 2] = 129                       # row 3, k 64..95 ×4
    c = mx.reference(a, b, sa, sb)
    assert c[0, 0] == 128 and c[3, 5] == 96 + 32 * 4
