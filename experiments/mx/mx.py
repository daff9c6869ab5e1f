"""Block-scaled (MX) matrix-core probes: gfx950's ``v_mfma_scale_f32_16x16x128_f8f6f4``.

An experiment kept next to gpumounter-amd, not part of it (moved out of ``gpumounter_amd/ops``
in round 5: the attach path validates a GPU with the wave64 liveness kernel only, and the
round-3 review ruled the fp8/fp4 pipes out of the product's scope). MI355X runs fp8 at twice
and fp4 at four times the bf16 MFMA rate. Library: ``libgm_mx.so`` next to this file
(``make -C native mx``).

* :func:`peak` — register-resident MX-MFMA throughput (fp8 or fp4) plus one sum per wave; the
  kernel is deterministic, so two runs (or two GPUs) must agree bit for bit;
* :func:`check_fp8` — one 16x16x128 tile of OCP e4m3 data with per-32-block E8M0 scales against
  a float64 host reference. The matrix core rounds inside the 128-term sum, so each output may
  differ by 2^-9 of its sum of |products|; a wrong lane map or scale is off by the order of the
  output itself.

Encodings (OCP, not MI300X's FNUZ): e4m3fn = 1 sign, 4 exponent (bias 7), 3 mantissa bits, no
infinities, 0x7F/0xFF NaN; e2m1 = 1 sign, 2 exponent (bias 1), 1 mantissa bit; E8M0 = 2^(e-127).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional, Tuple

import numpy as np

from gpumounter_amd import _native

HERE = os.path.dirname(os.path.abspath(__file__))
FMT = {"fp8": 0, "fp4": 4}


class MxError(RuntimeError):
    pass


_lib = []


def lib() -> C.CDLL:
    """``libgm_mx.so`` (``make -C native mx``), typed."""
    if not _lib:
        path = os.path.join(HERE, "libgm_mx.so")
        if not os.path.exists(path):
            raise MxError(f"{path} missing: make -C native mx")
        L = C.CDLL(path)
        L.gm_mx_peak.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                 C.POINTER(C.c_double)]
        L.gm_mx_peak_variant.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        L.gm_mx_tile.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
        L.gm_mx_strerror.argtypes = [C.c_int]
        L.gm_mx_strerror.restype = C.c_char_p
        _lib.append(L)
    return _lib[0]


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().gm_mx_strerror(rc).decode(errors="replace")
        raise MxError(f"{what}: {msg} ({rc})")


# ------------------------------------------------------------------------------ encodings
def e4m3_decode(code) -> np.ndarray:
    """OCP e4m3fn bytes → float64 (NaN for 0x7F/0xFF)."""
    c = np.asarray(code, np.uint8).astype(np.int64)
    s = np.where(c & 0x80, -1.0, 1.0)
    e = (c >> 3) & 0xF
    m = c & 0x7
    val = np.where(e == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * 2.0 ** (e - 7))
    val = np.where((c & 0x7F) == 0x7F, np.nan, val)
    return s * val


_E4M3_TABLE = e4m3_decode(np.arange(256, dtype=np.uint8))


def e4m3_encode(x: float) -> int:
    """The e4m3fn code of a value the format holds exactly (raises otherwise)."""
    hits = np.nonzero(_E4M3_TABLE == x)[0]
    if not len(hits):
        raise ValueError(f"{x} is not an e4m3 value")
    return int(hits[0])


def e8m0(code) -> np.ndarray:
    return 2.0 ** (np.asarray(code, np.float64) - 127)


# ------------------------------------------------------------------------------ lane maps
# v_mfma_scale_f32_16x16x128_f8f6f4 with 8-bit operands, measured on MI355X with exact one-hot
# data (round-3 probes, profiles/r3_mx/: rows and the A↔B pairing, which lane's scale
# multiplies each byte, which fixes the true k). Lane l holds row (A) / column (B) l & 15; its
# bytes 0-15 are k = 16 (l >> 4) + j and bytes 16-31 are k = 64 + 16 (l >> 4) + (j - 16), so one
# lane spans two 32-wide scale blocks. The E8M0 scale of row/column r, block s (k in
# [32 s, 32 s + 32)) is read from lane r + 16 s. C/D: col = l & 15, row = 4 (l >> 4) + reg — the
# dtype-independent gfx950 16x16 map.
def k_index(lane: int, byte: int) -> int:
    h = lane >> 4
    return 16 * h + byte if byte < 16 else 64 + 16 * h + (byte - 16)


_K = np.array([[k_index(ln, j) for j in range(32)] for ln in range(64)])


def a_lanes(a: np.ndarray) -> np.ndarray:
    """A [16 rows][128 k] → per-lane register images [64 lanes][32 bytes]."""
    return np.ascontiguousarray(np.stack([a[ln & 15, _K[ln]] for ln in range(64)]))


def b_lanes(b: np.ndarray) -> np.ndarray:
    """B [128 k][16 cols] → per-lane register images [64 lanes][32 bytes]."""
    return np.ascontiguousarray(np.stack([b[_K[ln], ln & 15] for ln in range(64)]))


def scale_lanes(s: np.ndarray) -> np.ndarray:
    """Block scales [16 rows or cols][4 blocks] → the 64 per-lane scale bytes."""
    return np.array([s[ln & 15, ln >> 4] for ln in range(64)], np.uint8)


def c_from_lanes(c: np.ndarray) -> np.ndarray:
    """Per-lane accumulators [64][4] → C [16 rows][16 cols]."""
    out = np.zeros((16, 16), c.dtype)
    for ln in range(64):
        for r in range(4):
            out[4 * (ln >> 4) + r, ln & 15] = c[ln, r]
    return out


# ------------------------------------------------------------------------------ GPU calls
def tile(dev: int, afrag: np.ndarray, bfrag: np.ndarray, sa: np.ndarray, sb: np.ndarray,
         fmt: str = "fp8") -> np.ndarray:
    """One MX-MFMA on raw per-lane images (64×32 bytes each, 64 scale bytes each) → [64][4]."""
    a = np.ascontiguousarray(afrag, np.uint8)
    b = np.ascontiguousarray(bfrag, np.uint8)
    sa = np.ascontiguousarray(sa, np.uint8)
    sb = np.ascontiguousarray(sb, np.uint8)
    if a.shape != (64, 32) or b.shape != (64, 32) or sa.shape != (64,) or sb.shape != (64,):
        raise ValueError("afrag/bfrag must be 64×32 bytes, sa/sb 64 bytes")
    c = np.zeros((64, 4), np.float32)
    _check(lib().gm_mx_tile(dev, FMT[fmt], a.ctypes.data, b.ctypes.data,
                                            sa.ctypes.data, sb.ctypes.data, c.ctypes.data),
           "mx tile")
    return c


BEST_VARIANT = {"fp8": 1, "fp4": 2}   # profiles/r3_mx/sweep.json


def peak(dev: int, fmt: str = "fp8", iters: int = 10000, blocks_per_cu: int = 8,
         variant: Optional[int] = None) -> Tuple[float, np.ndarray]:
    """(dense TF/s, per-wave sums) of the register-resident MX-MFMA loop. variant 0: 16x16x128
    × 8 chains; 1: 32x32x64 × 4; 2: 32x32x64 × 8; None: the measured best for ``fmt``."""
    variant = BEST_VARIANT[fmt] if variant is None else variant
    p = _native.ProbeProps()
    _check(_native.probe().gm_probe_props(dev, C.byref(p)), "props")
    n = p.cu_count * blocks_per_cu * 4
    sums = np.zeros(n, np.float32)
    t = C.c_double(0)
    _check(lib().gm_mx_peak_variant(dev, FMT[fmt], variant, iters, blocks_per_cu,
                                        sums.ctypes.data, n, C.byref(t)), "mx peak")
    return t.value, sums


def reference(a: np.ndarray, b: np.ndarray, sa: np.ndarray, sb: np.ndarray) -> np.ndarray:
    """C = Σ_k decode(A)·2^(sA−127) · decode(B)·2^(sB−127) in float64; sa [16 rows][4 blocks],
    sb [16 cols][4 blocks]."""
    av = e4m3_decode(a) * np.repeat(e8m0(sa), 32, axis=1)          # [16][128]
    bv = e4m3_decode(b) * np.repeat(e8m0(sb), 32, axis=1).T        # [128][16]
    return av @ bv


def check_fp8(dev: int, seed: int = 0) -> Dict:
    """Random e4m3 A [16×128], B [128×16] (|x| ≤ 8, no NaN) with random E8M0 block scales in
    2^-4…2^4 through one MX-MFMA; compared with :func:`reference`."""
    rng = np.random.default_rng(seed)
    finite = np.array([c for c in range(256) if (c & 0x7F) != 0x7F and
                       abs(_E4M3_TABLE[c]) <= 8.0], np.uint8)
    a = rng.choice(finite, size=(16, 128))
    b = rng.choice(finite, size=(128, 16))
    sa = rng.integers(123, 132, size=(16, 4)).astype(np.uint8)
    sb = rng.integers(123, 132, size=(16, 4)).astype(np.uint8)
    got = c_from_lanes(tile(dev, a_lanes(a), b_lanes(b), scale_lanes(sa), scale_lanes(sb)))
    want = reference(a, b, sa, sb)
    # the matrix core does not keep every bit of the 128-term sum (measured: ≈2^-13 of the sum
    # of |products|); a wrong lane map or scale is off by the order of the result itself
    bound = reference(np.where(a & 0x80, a ^ 0x80, a), np.where(b & 0x80, b ^ 0x80, b), sa, sb)
    err = np.abs(got.astype(np.float64) - want)
    worst = float(np.max(err / np.maximum(bound, 1e-30)))
    return {"max_abs_err": float(np.max(err)), "ref_scale": float(np.max(np.abs(want))),
            "max_err_over_abs_sum": worst, "ok": worst <= 2.0 ** -9}


def burn_in(dev: int, seconds: float = 10.0, fmt: str = "fp8") -> Dict:
    """Sustained MX-pipe load for ``seconds``: every launch's per-wave sums are compared bit for
    bit with the first launch's (the kernel is deterministic — a round-3 probe measured 0
    differing waves over thousands), so any ``mismatches`` is silent data corruption on the fp8 /
    fp4 matrix path; ``tflops`` the sustained rate (throttling shows up as a low number)."""
    import time
    first = None
    bad, runs, rates = 0, 0, []
    end = time.monotonic() + seconds
    while time.monotonic() < end or runs == 0:
        t, sums = peak(dev, fmt)
        u = sums.view(np.uint32)
        if first is None:
            first = u.copy()
        else:
            bad += int(np.sum(u != first))
        rates.append(t)
        runs += 1
    return {"device": dev, "fmt": fmt, "seconds": seconds, "launches": runs,
            "tflops": float(np.median(rates)), "mismatches": bad, "ok": bad == 0}
