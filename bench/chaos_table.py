#!/usr/bin/env python3
"""The round's sweep table for profiles/r6_chaos/README.md: every ``<dir>/runs.jsonl`` with the
commit it ran at, and the totals.

    python bench/chaos_table.py profiles/r6_chaos > /tmp/table.md
"""
import json
import os
import sys

# the frozen worktree's commit per sweep (a GPU box run gets no git metadata: the tree sent)
COMMITS = {"sweep1": "≥ `dfe7c34`", "sweep2": "≥ `dfe7c34`", "sweep3": "`f281d3f`",
           "sweep4": "`f281d3f`", "sweep5": "`f281d3f`", "sweep6": "`3155cd6`",
           "sweep7": "`3155cd6`", "sweep8": "`61b3c08`", "sweep9": "`61b3c08`",
           "sweep10": "`7840df0`", "sweep11": "`7840df0`", "sweep12": "`0a02c8c`",
           "sweep13": "`0a02c8c`", "sweep14": "`197ce4f`", "sweep15": "`197ce4f`",
           "sweep16": "`197ce4f`", "sweep17": "`197ce4f`",
           "sweep18": "`0fded3c`", "sweep19": "`ec95933`", "sweep20": "`6fef154`",
           "box1": "`47fda63`",
           "box2": "`c89abea`", "box3": "`7de522a`", "box4": "`9880c89`", "box5": "`3bfbd67`",
           "box6": "`197ce4f`", "box7": "`197ce4f`", "box8": "`bbeb156`",
           "box9": "`f9547fe`", "box10": "`ec95933`",
           "box11": "`d797c3e`", "box12": "`be874bf`",
           "box13": "`28b1cd0`", "box14": "`046af1b`",
           "box15": "`756693b`"}


def main(root: str) -> int:
    names = sorted((d for d in os.listdir(root) if os.path.exists(f"{root}/{d}/runs.jsonl")),
                   key=lambda d: (d.startswith("box"), int("".join(c for c in d if c.isdigit()))))
    print("| sweep | where | commit | modes | seeds | runs | worker / master kills | kubelet "
          "restarts | container restarts / Pod re-creations | preemptors / standbys preempted "
          "| ops ok | invariant violations (or failed starts) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    keys = ("worker_kills", "master_kills", "kubelet_restarts", "container_restarts",
            "pod_recreates", "preemptors", "ops_ok")
    tot = dict.fromkeys(keys + ("runs", "standby", "bad"), 0)
    for d in names:
        rs = [json.loads(ln) for ln in open(f"{root}/{d}/runs.jsonl") if ln.strip()]
        g = {k: sum(int(r.get(k) or 0) for r in rs) for k in keys}
        bad = sum(int(r.get("invariant_violations") or 0) for r in rs) + \
            sum(1 for r in rs if r.get("error"))
        standby = sum((r.get("preempted") or {}).get("standby", 0) for r in rs)
        seeds = sorted({int(r["seed"]) for r in rs})
        print(f"| `{d}` | {'GPU box' if d.startswith('box') else 'here'} | "
              f"{COMMITS.get(d, '?')} | {len({r['mode'] for r in rs})} | "
              f"{seeds[0]}–{seeds[-1]} | {len(rs)} | {g['worker_kills']} / {g['master_kills']} "
              f"| {g['kubelet_restarts']} | {g['container_restarts']} / {g['pod_recreates']} | "
              f"{g['preemptors']} / {standby} | {g['ops_ok']} | **{bad}** |")
        for k in keys:
            tot[k] += g[k]
        tot["runs"] += len(rs)
        tot["standby"] += standby
        tot["bad"] += bad
    print(f"| **total** | | | | | **{tot['runs']}** | {tot['worker_kills']} / "
          f"{tot['master_kills']} | {tot['kubelet_restarts']} | {tot['container_restarts']} / "
          f"{tot['pod_recreates']} | {tot['preemptors']} / {tot['standby']} | {tot['ops_ok']} "
          f"| {tot['bad']} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "profiles/r6_chaos"))
