#!/usr/bin/env python3
"""Markdown rows for chaos sweeps: one row per ``<dir>/runs.jsonl`` (bench/chaos_sweep.py).

    python bench/sweep_table.py profiles/r6_chaos/sweep1 profiles/r6_chaos/sweep2 ...
"""
import json
import sys


def main(dirs) -> int:
    print("| sweep | seeds | runs | worker / master kills | kubelet restarts | container "
          "restarts / Pod re-creations | preemptors / standbys preempted | ops ok | invariant "
          "violations |")
    print("|---|---|---|---|---|---|---|---|---|")
    total = 0
    for d in dirs:
        rows = [json.loads(ln) for ln in open(f"{d}/runs.jsonl") if ln.strip()]

        def tot(k):
            return sum(int(r.get(k) or 0) for r in rows)
        seeds = sorted({int(r["seed"]) for r in rows})
        v = tot("invariant_violations")
        standby = sum((r.get("preempted") or {}).get("standby", 0) for r in rows)
        total += v
        print(f"| `{d.rstrip('/').split('/')[-1]}` | {seeds[0]}–{seeds[-1]} | {len(rows)} | "
              f"{tot('worker_kills')} / {tot('master_kills')} | {tot('kubelet_restarts')} | "
              f"{tot('container_restarts')} / {tot('pod_recreates')} | "
              f"{tot('preemptors')} / {standby} | "
              f"{tot('ops_ok')} | "
              f"**{v}** |")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
