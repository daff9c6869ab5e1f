"""Python side of the gfx950 post-attach validation kernels (native/hip/gm_probe.hip; the burn-in
GEMM in native/hip/gm_gemm.hip).

An attach is only useful if the tenant can actually run work on the GPU. After the node operations
succeed, a tenant-side agent (or the bench ranks) call :func:`verify` on the newly attached devices:
a wave64 liveness kernel (every lane writes, a 64-lane shuffle reduction and a 64-bit ballot are
checked), and optionally an HBM3E stream, an MFMA bf16 peak and an MFMA GEMM numerics check.
No silent fallback: if ``libgm_probe.so`` is missing or HIP fails, this raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional

from gpumounter_amd import _native


class ProbeError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _native.probe().gm_probe_strerror(rc).decode(errors="replace")
        raise ProbeError(f"{what}: hip error {rc} ({msg})")


def device_count() -> int:
    n = C.c_int(0)
    _check(_native.probe().gm_probe_device_count(C.byref(n)), "hipGetDeviceCount")
    return n.value


def props(dev: int) -> Dict:
    p = _native.ProbeProps()
    _check(_native.probe().gm_probe_props(dev, C.byref(p)), "props")
    return {"name": p.name.decode(), "gcn_arch": p.gcn_arch.decode(),
            "pci_bus_id": p.pci_bus_id.decode().lower(), "cu_count": p.cu_count,
            "warp_size": p.warp_size, "total_mem": p.total_mem,
            "lds_per_block": p.lds_per_block, "clock_khz": p.clock_khz}


def find_device(bdf: str) -> int:
    """HIP device index of the GPU at PCI address ``bdf`` (-1 if not visible)."""
    d = C.c_int(-1)
    _check(_native.probe().gm_probe_find_device(bdf.encode(), C.byref(d)), "find_device")
    return d.value


def quick(dev: int) -> float:
    """Liveness kernel; returns launch→readback µs. Raises if the wave64 checks fail."""
    ok, us = C.c_int(0), C.c_double(0)
    _check(_native.probe().gm_probe_quick(dev, C.byref(ok), C.byref(us)), "quick probe")
    if not ok.value:
        raise ProbeError(f"device {dev}: liveness kernel produced wrong results")
    return us.value


def hbm_gbps(dev: int, nbytes: int = 1 << 30, iters: int = 10) -> float:
    g = C.c_double(0)
    _check(_native.probe().gm_probe_hbm_copy(dev, nbytes, iters, C.byref(g)), "hbm copy")
    return g.value


def hbm_read_gbps(dev: int, nbytes: int = 1 << 30, iters: int = 10,
                  blocks_per_cu: int = 2) -> float:
    g = C.c_double(0)
    _check(_native.probe().gm_probe_hbm_read(dev, nbytes, iters, blocks_per_cu, C.byref(g)),
           "hbm read")
    return g.value


def mfma_tflops(dev: int, iters: int = 20000) -> float:
    t = C.c_double(0)
    _check(_native.probe().gm_probe_mfma_peak(dev, iters, C.byref(t)), "mfma peak")
    return t.value


def gemm_check(dev: int, m: int = 256, n: int = 256, k: int = 256) -> Dict[str, float]:
    err, scale = C.c_double(0), C.c_double(0)
    _check(_native.probe().gm_probe_gemm_check(dev, m, n, k, C.byref(err), C.byref(scale)),
           "gemm check")
    return {"max_abs_err": err.value, "ref_scale": scale.value}


def gemm_bf16(a, b, out=None, stream=None):
    """C(fp32) = A(bf16) @ B(bf16) on MFMA for torch tensors on a HIP device.

    Shapes: A [M,K], B [K,N] contiguous; M, N multiples of 64 and K a multiple of 32.
    """
    import torch

    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise ProbeError("gemm_bf16 expects bf16 inputs")
    if not (a.is_contiguous() and b.is_contiguous()):
        raise ProbeError("gemm_bf16 expects contiguous inputs")
    m, k = a.shape
    k2, n = b.shape
    if k != k2 or m % 64 or n % 64 or k % 32:
        raise ProbeError(f"unsupported shape A{tuple(a.shape)} B{tuple(b.shape)}")
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    s = stream if stream is not None else torch.cuda.current_stream(a.device)
    with torch.cuda.device(a.device):
        _check(_native.probe().gm_probe_gemm_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                                  m, n, k, C.c_void_p(s.cuda_stream)),
               "gemm_bf16")
    return out


def gemm_nt(a, bt, out=None, stream=None, variant: Optional[int] = None):
    """C(bf16) = A @ Btᵀ for bf16 torch tensors on a HIP device: the 256²-tile
    global_load_lds MFMA GEMM (gm_probe_gemm_nt). Shapes: A [M,K], Bt [N,K] contiguous
    (both K-major); M, N multiples of 256 and K a multiple of 64. ``variant`` picks a schedule
    (0: per-k-step fragment reads, 1: whole K-tile of reads up front, 2: quadrant phases,
    3: V1 on 32x32x16, 4: 4 waves × 128², 5: local-read prefetch across the barrier, 6: V4 on
    V5's schedule with buffer_load-to-LDS staging, 7: V5 with buffer_load-to-LDS staging, 8: V5 with a DPP-transposed 8-byte-store epilogue, 9: V2 with register prefetch across phases;
    default: the fastest measured, 5 — profiles/history/r1_gemm)."""
    import torch

    if a.dtype != torch.bfloat16 or bt.dtype != torch.bfloat16:
        raise ProbeError("gemm_nt expects bf16 inputs")
    if not (a.is_contiguous() and bt.is_contiguous()):
        raise ProbeError("gemm_nt expects contiguous inputs")
    m, k = a.shape
    n, k2 = bt.shape
    if k != k2 or m % 256 or n % 256 or k % 64:
        raise ProbeError(f"unsupported shape A{tuple(a.shape)} Bt{tuple(bt.shape)}")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ProbeError("gemm_nt: out must be a contiguous bf16 [M,N] tensor")
    s = stream if stream is not None else torch.cuda.current_stream(a.device)
    with torch.cuda.device(a.device):
        lib = _native.probe()
        ptrs = (a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k, C.c_void_p(s.cuda_stream))
        rc = (lib.gm_probe_gemm_nt(*ptrs) if variant is None
              else lib.gm_probe_gemm_nt_variant(variant, *ptrs))
        _check(rc, "gemm_nt")
    return out


def gemm_tflops(dev: int, m: int = 8192, n: int = 8192, k: int = 8192, iters: int = 10) -> float:
    """Dense bf16 TF/s of the 256²-tile GEMM on uniform [-1,1) operands (burn-in load)."""
    t = C.c_double(0)
    _check(_native.probe().gm_probe_gemm_nt_tflops(dev, m, n, k, iters, C.byref(t)),
           "gemm tflops")
    return t.value


def burn_in(dev: int, seconds: float = 10.0, n: int = 8192) -> Dict:
    """Sustained-load check of an attached GPU: back-to-back n³ bf16 GEMMs for ``seconds``,
    each compared bit-for-bit with the first result (the kernel is deterministic). Any
    ``mismatches`` means silent data corruption. ``tflops`` is the sustained rate, so
    throttling shows up as a low number."""
    tf, bad, it = C.c_double(0), C.c_uint64(0), C.c_int(0)
    _check(_native.probe().gm_probe_burn_in(dev, n, seconds, C.byref(tf), C.byref(bad),
                                            C.byref(it)), "burn-in")
    return {"device": dev, "n": n, "seconds": seconds, "iterations": it.value,
            "tflops": tf.value, "mismatches": bad.value, "ok": bad.value == 0}


def p2p(dev_a: int, dev_b: int, nbytes: int = 256 << 20, iters: int = 10) -> Dict:
    can, g = C.c_int(0), C.c_double(0)
    _check(_native.probe().gm_probe_p2p(dev_a, dev_b, nbytes, iters, C.byref(can), C.byref(g)),
           "p2p")
    return {"src": dev_a, "dst": dev_b, "peer_access": bool(can.value), "gbps": g.value}


@dataclass
class VerifyResult:
    device: int
    bdf: str
    quick_us: float
    gcn_arch: str
    hbm_gbps: Optional[float] = None
    hbm_read_gbps: Optional[float] = None
    mfma_tflops: Optional[float] = None
    gemm_max_abs_err: Optional[float] = None
    gemm_tflops: Optional[float] = None

    def to_dict(self) -> Dict:
        return asdict(self)


def verify(bdfs: List[str], full: bool = False) -> List[VerifyResult]:
    """Run the validation on each attached GPU (by PCI address)."""
    out = []
    for bdf in bdfs:
        dev = find_device(bdf)
        if dev < 0:
            raise ProbeError(f"attached GPU {bdf} is not visible to HIP in this process")
        pr = props(dev)
        r = VerifyResult(dev, bdf, quick(dev), pr["gcn_arch"])
        if full:
            r.hbm_gbps = hbm_gbps(dev)
            r.hbm_read_gbps = hbm_read_gbps(dev)
            r.mfma_tflops = mfma_tflops(dev)
            r.gemm_max_abs_err = gemm_check(dev)["max_abs_err"]
            r.gemm_tflops = gemm_tflops(dev, 4096, 4096, 4096, 10)
        out.append(r)
    return out
