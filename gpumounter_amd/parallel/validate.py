"""Tenant-side check after an attach: ``python -m gpumounter_amd.parallel.validate``.

Run inside the pod once GPUs were hot-mounted. It answers the questions a tenant has before
starting a job on them — the reference offers nothing here:

1. every visible GPU runs a gfx950 kernel (wave64 liveness probe, :mod:`gpumounter_amd.ops.probe`);
2. every pair has peer access and xGMI-class copy bandwidth (:func:`collectives.xgmi_matrix`);
3. RCCL works across all of them: one process per GPU, ``torch.distributed`` with backend
   ``nccl`` (RCCL on ROCm), a checked bf16 all-reduce with ring bus bandwidth
   (:func:`collectives.allreduce_check`);
4. optionally (``--burn-in SECONDS``) all GPUs under sustained MFMA load at once, each
   result bit-compared with the first: bf16 GEMMs for SECONDS (:func:`probe.burn_in`). Catches
   silent data corruption and throttling that a short probe misses.

Prints one JSON document; exit code 0 only if every check passed. ``--cpu-ranks N`` runs step 3
with N gloo ranks on the CPU (hermetic tests).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Dict, List


def _rank_main(rank: int, world: int, cpu: bool, numel: int, out_dir: str) -> None:
    import torch
    import torch.distributed as dist

    from gpumounter_amd.parallel.collectives import allreduce_check

    # file:// rendezvous in the run's own directory: no TCP port picked ahead of time (another
    # process can take a port between the pick and rank 0's bind)
    rdv = "file://" + os.path.join(out_dir, "rendezvous")
    if cpu:
        dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(rank)
        dev = torch.device("cuda", rank)
        dist.init_process_group("nccl", init_method=rdv, rank=rank, world_size=world,
                                device_id=dev)
    try:
        res = allreduce_check(numel=numel, device=dev)
    finally:
        dist.destroy_process_group()
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as fh:
        json.dump(res, fh)


def run_allreduce(world: int, cpu: bool, numel: int) -> List[Dict]:
    import tempfile

    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory(prefix="gm-validate-") as out_dir:
        mp.spawn(_rank_main, args=(world, cpu, numel, out_dir), nprocs=world, join=True)
        res = []
        for r in range(world):
            with open(os.path.join(out_dir, f"rank{r}.json")) as fh:
                res.append(json.load(fh))
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gpumounter_amd.parallel.validate")
    ap.add_argument("--cpu-ranks", type=int, default=0,
                    help="skip the GPU checks; all-reduce over N gloo ranks on the CPU")
    ap.add_argument("--numel", type=int, default=1 << 24, help="all-reduce elements (bf16)")
    ap.add_argument("--no-p2p", action="store_true")
    ap.add_argument("--burn-in", type=float, default=0.0, metavar="SECONDS",
                    help="then load every GPU at once with bit-checked GEMMs for SECONDS")
    args = ap.parse_args(argv)
    report: Dict = {"ok": True}
    if args.cpu_ranks:
        world = args.cpu_ranks
    else:
        from gpumounter_amd.ops import probe
        from gpumounter_amd.parallel.collectives import xgmi_matrix

        n = probe.device_count()
        if n == 0:
            print(json.dumps({"ok": False, "error": "no GPU visible (nothing attached?)"}))
            return 1
        devs = list(range(n))
        report["gpus"] = [{"device": d, "bdf": probe.props(d)["pci_bus_id"],
                           "arch": probe.props(d)["gcn_arch"], "quick_us": probe.quick(d)}
                          for d in devs]
        if n > 1 and not args.no_p2p:
            m = xgmi_matrix(devs)
            report["p2p"] = m
            report["ok"] &= all(all(row) for row in m["peer"])
        world = n
    ranks = run_allreduce(world, bool(args.cpu_ranks), args.numel)
    report["allreduce"] = {"world": world, "ok": all(r["ok"] for r in ranks),
                           "ms": max(r["ms"] for r in ranks),
                           "busbw_gbps": min(r["busbw_gbps"] for r in ranks),
                           "bytes": ranks[0]["bytes"]}
    report["ok"] &= report["allreduce"]["ok"]
    if args.burn_in and not args.cpu_ranks:
        from concurrent.futures import ThreadPoolExecutor

        from gpumounter_amd.ops import probe

        # all GPUs at once (shared power/thermal envelope); ctypes drops the GIL in the call
        with ThreadPoolExecutor(max_workers=world) as ex:
            burn = list(ex.map(lambda d: probe.burn_in(d, args.burn_in), range(world)))
        report["burn_in"] = burn
        report["ok"] &= all(b["ok"] for b in burn)
    print(json.dumps(report))
    return 0 if report["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
