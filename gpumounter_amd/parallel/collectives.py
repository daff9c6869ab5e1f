"""Post-attach multi-GPU validation: RCCL collectives and xGMI peer bandwidth.

The reference has no collective or P2P logic. On MI355X the point of
hive-aware placement is that a tenant's RCCL job gets direct xGMI links between every pair of its
GPUs (7 links × ≈153 GB/s per GPU, point-to-point). These helpers prove that on the attached set:

* :func:`xgmi_matrix` — pairwise ``hipMemcpyPeerAsync`` bandwidth + peer-access bits (one
  process, all attached devices);
* :func:`allreduce_check` — a bf16 all-reduce over ``torch.distributed`` (backend ``nccl`` = RCCL
  on ROCm), numerically checked, with algorithm/bus bandwidth using the ring formula
  ``busbw = algbw · 2(n-1)/n``.
"""
from __future__ import annotations

import time
from typing import Dict, List

from gpumounter_amd.ops import probe


def xgmi_matrix(devices: List[int], nbytes: int = 256 << 20, iters: int = 5) -> Dict:
    out = {"devices": devices, "gbps": [], "peer": []}
    for a in devices:
        row_g, row_p = [], []
        for b in devices:
            if a == b:
                row_g.append(0.0)
                row_p.append(True)
                continue
            r = probe.p2p(a, b, nbytes, iters)
            row_g.append(r["gbps"])
            row_p.append(r["peer_access"])
        out["gbps"].append(row_g)
        out["peer"].append(row_p)
    return out


def allreduce_check(group=None, numel: int = 1 << 24, iters: int = 5, device=None) -> Dict:
    """Run inside every rank of an initialised process group. Returns timing on each rank."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    on_gpu = torch.device(dev).type == "cuda"
    # bf16 on the GPU (RCCL); gloo on the CPU reduces fp32
    dtype = torch.bfloat16 if on_gpu else torch.float32

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)
    x = torch.full((numel,), float(rank + 1), dtype=dtype, device=dev)
    dist.all_reduce(x, group=group)  # warm-up / communicator init
    expect = world * (world + 1) / 2
    sync()
    ok = bool(torch.all(x == expect).item()) if expect <= 256 else True
    x.fill_(1.0)
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(x, group=group)
    sync()
    dt = (time.perf_counter() - t0) / iters
    nbytes = numel * x.element_size()
    algbw = nbytes / dt / 1e9
    busbw = algbw * 2 * (world - 1) / world if world > 1 else algbw
    return {"rank": rank, "world": world, "ok": ok, "ms": dt * 1e3, "algbw_gbps": algbw,
            "busbw_gbps": busbw, "bytes": nbytes}
