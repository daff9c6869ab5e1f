#!/usr/bin/env python3
"""Run the every-mode chaos sweep (profiles/r4_chaos_full/README.md, "every mode") over seeds.

    python bench/chaos_sweep.py --seeds 200 201 --jobs 3 --out profiles/r5_chaos/sweep1

Each (mode, seed) is one ``bench/configs.py chaos`` process with the round-4 base flags (process
deployment, worker/master/kubelet kills, 10 % apiserver faults, stage faults) plus the mode's
own; its JSON line goes to ``<out>/runs.jsonl`` keyed ``<mode><seed>``, its logs to
``<out>/logs/<mode><seed>/``. Prints one summary line per run and the total of invariant
violations at the end (exit status 1 if there are any).
"""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = ["--rounds", "100", "--kill-every", "5", "--master-kill-every", "3",
        "--api-fault-rate", "0.1", "--kubelet-restart-every", "7", "--reconcile-period", "30",
        "--faults", "--deploy", "processes"]
CHURN = ["--restart-rate", "0.3", "--recreate-rate", "0.1"]


def _commit() -> str:
    """The code under test (the frozen worktree's HEAD); "" outside git (a GPU box copy)."""
    try:
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"],
                              capture_output=True, text=True, timeout=10).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        return ""


COMMIT = _commit()
MODES = {
    "f": CHURN,
    "pool": CHURN + ["--warm-pool", "2"],
    "dra": CHURN + ["--gpu-api", "dra"],
    "pl": CHURN + ["--warm-pool", "2", "--lease-rate", "0.4"],
    "dpl": CHURN + ["--gpu-api", "dra", "--warm-pool", "3", "--lease-rate", "0.3"],
    "bp": ["--busy", "--warm-pool", "3"],
    "v1pl": CHURN + ["--cgroup", "v1", "--warm-pool", "2", "--lease-rate", "0.3"],
    "rpl": CHURN + ["--alloc-policy", "random", "--warm-pool", "2", "--lease-rate", "0.3"],
    "hpl": CHURN + ["--placement", "hint", "--warm-pool", "2", "--lease-rate", "0.3"],
    "tpr": ["--restart-rate", "0.2", "--placement", "trim", "--warm-pool", "2",
            "--lease-rate", "0.3"],
    # round 6: idle standbys at the low pool class; every attach that needs them yields them
    "lpl": CHURN + ["--warm-pool", "2", "--pool-priority-class", "gpumounter-standby",
                    "--lease-rate", "0.3"],
    # round 6: a higher-priority Pod that wants node-0's GPUs arrives and leaves between
    # rounds; the scheduler preempts the lowest-priority pods it can (standbys, tenants)
    "pre": CHURN + ["--warm-pool", "2", "--pool-priority-class", "gpumounter-standby",
                    "--preempt-rate", "0.5"],
    "pre0": CHURN + ["--preempt-rate", "0.5"],
    # placeholders bound to the node at creation (no scheduling cycle), racing preemptors the
    # scheduler binds, with a warm pool and leases
    "dir": CHURN + ["--placeholder-binding", "direct", "--preempt-rate", "0.5",
                    "--warm-pool", "2", "--lease-rate", "0.3"],
    # a kubelet that frees a deleted Pod's devices 50 ms after the DELETE: attaches and pool
    # refills right after a detach are refused at admission and retried
    "td": CHURN + ["--latency", "teardown", "--warm-pool", "2", "--pool-priority-class",
                   "gpumounter-standby", "--lease-rate", "0.3"],
    "tdd": CHURN + ["--latency", "teardown", "--placeholder-binding", "direct",
                    "--preempt-rate", "0.5"],
    # the kubelet's checkpoint keeps deleted Pods until the next Allocate, as a real one does
    "lz": CHURN + ["--lazy-checkpoint", "--latency", "teardown", "--warm-pool", "2",
                   "--lease-rate", "0.3"],
}


def one(mode: str, seed: int, out: str, timeout: float) -> dict:
    key = f"{mode}{seed}"
    logs = os.path.join(out, "logs", key)
    os.makedirs(logs, exist_ok=True)
    argv = [sys.executable, os.path.join(ROOT, "bench", "configs.py"), "chaos", *BASE,
            *MODES[mode], "--seed", str(seed), "--log-dir", logs]
    t0 = time.time()
    try:
        p = subprocess.run(argv, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        res = json.loads(lines[-1]) if lines else {"error": p.stderr[-2000:], "rc": p.returncode}
    except subprocess.TimeoutExpired:
        res = {"error": f"timed out after {timeout:g}s"}
    res.update(run=key, mode=mode, seed=seed, wall_s=round(time.time() - t0, 1),
               argv=argv[2:], commit=COMMIT)
    if res.get("invariant_violations") == 0 and "error" not in res:
        shutil.rmtree(logs, ignore_errors=True)     # a clean run's logs are not kept
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", required=True)
    ap.add_argument("--modes", nargs="+", default=list(MODES), choices=list(MODES))
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("--out", required=True)
    ap.add_argument("--timeout", type=float, default=1800.0)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    todo = [(m, s) for s in args.seeds for m in args.modes]
    bad = 0
    with cf.ThreadPoolExecutor(args.jobs) as ex, \
            open(os.path.join(args.out, "runs.jsonl"), "a") as fh:
        futs = {ex.submit(one, m, s, args.out, args.timeout): (m, s) for m, s in todo}
        for f in cf.as_completed(futs):
            r = f.result()
            fh.write(json.dumps(r) + "\n")
            fh.flush()
            v = r.get("invariant_violations")
            bad += 1 if v is None else int(v)
            print(f"{r['run']:>10}  violations={v}  ops_ok={r.get('ops_ok')}  "
                  f"{r['wall_s']}s  {r.get('error', '')[:200]}", flush=True)
    print(f"total invariant violations (or failed runs): {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
