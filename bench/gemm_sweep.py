"""Burn-in GEMM (gm_probe_gemm_nt, 256² tile, global_load_lds) vs torch.matmul on one MI355X.

Same uniform [-1, 1) bf16 operands for both (zero-filled operands overstate a GEMM by ≈20 %
through DVFS, cdna_hip_programming.md §5.4 rule 25). Variants are timed in interleaved rounds in
one process (rule 24); the JSON reports median and best TF/s per variant and shape, plus the
max error of ours against torch's fp32 product on a 1024³ slice. Run on the GPU box:
``python bench/gemm_sweep.py [--rounds 5] [--variants 1,5]``.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gpumounter_amd import _native  # noqa: E402
from gpumounter_amd.ops import probe  # noqa: E402


def ours(variant, a, bt, c):
    lib = _native.probe()
    m, k = a.shape
    n = bt.shape[0]
    rc = lib.gm_probe_gemm_nt_variant(variant, a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k,
                                      C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    return c


def timed(fn, iters):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


VARIANTS = (1, 5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--variants", default=",".join(map(str, VARIANTS)),
                    help="schedules of gm_probe_gemm_nt_variant to time (1 or 5; 5 = default)")
    args = ap.parse_args()
    variants_sel = [int(v) for v in args.variants.split(",") if v]
    out = {"device": torch.cuda.get_device_name(0), "TFLOPs": {}, "numerics": {}}
    g = torch.Generator(device="cuda").manual_seed(0)
    for n in [int(x) for x in args.sizes.split(",")]:
        a = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        b = bt.t().contiguous()
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        variants = {f"gm_gemm_nt_v{v}": (lambda v=v: ours(v, a, bt, c)) for v in variants_sel}
        variants.update({
            "torch_nt": lambda: torch.matmul(a, bt.t(), out=c),
            "torch_nn": lambda: torch.matmul(a, b, out=c),
        })
        for fn in variants.values():
            fn()
        torch.cuda.synchronize()
        iters = max(3, int(2e13 / (2 * n ** 3)))
        res = {k: [] for k in variants}
        for _ in range(args.rounds):
            for k, fn in variants.items():
                res[k].append(2 * n ** 3 / timed(fn, iters) / 1e12)
        out["TFLOPs"][str(n)] = {k: {"median": round(statistics.median(v), 1),
                                     "best": round(max(v), 1)} for k, v in res.items()}
        print(json.dumps({str(n): out["TFLOPs"][str(n)]}), file=sys.stderr, flush=True)
        del a, bt, b, c
    a = (torch.rand(1024, 1024, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(1024, 1024, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ bt.float().t()
    checks = {f"gm_gemm_nt_v{v}": (lambda v=v: ours(v, a, bt, torch.empty_like(a)))
              for v in variants_sel}
    checks["torch_nt"] = lambda: torch.matmul(a, bt.t())
    for k, fn in checks.items():
        err = (fn().float() - ref).abs().max().item()
        out["numerics"][k] = {"max_abs_err_vs_fp32": err,
                              "ref_max": ref.abs().max().item()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
