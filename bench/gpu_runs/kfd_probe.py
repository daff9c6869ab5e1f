"""What KFD's process table and amdsmi's process list report for one GPU tenant, next to what
the tenant sees of itself (PID namespace evidence for busy detection; VERDICT r5 missing #2).

Order matters: the child opens the GPU first; this parent reads sysfs, and only then opens
amdsmi (it never execs after touching the GPU). Writes gpurun_out/kfd_probe.json.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

KFD = "/sys/class/kfd/kfd/proc"
CHILD = r"""
import os, sys, torch
x = torch.empty(256 << 20, dtype=torch.uint8, device="cuda:0"); torch.cuda.synchronize()
st = open("/proc/self/status").read().splitlines()
ns = [l for l in st if l.startswith("NSpid")][0].split()[1:]
print(os.getpid(), " ".join(ns), flush=True)
sys.stdin.read()
"""


def listing() -> list:
    try:
        return sorted(os.listdir(KFD), key=lambda s: (len(s), s))
    except OSError as e:
        return [f"error: {e}"]


def entry(pid: str) -> dict:
    out = {}
    base = os.path.join(KFD, pid)
    for root, dirs, files in os.walk(base):
        for f in sorted(files):
            p = os.path.join(root, f)
            rel = os.path.relpath(p, base)
            try:
                with open(p, "r", errors="replace") as fh:
                    out[rel] = fh.read(200).strip()
            except OSError as e:
                out[rel] = f"error: {e.strerror}"
        if root.count(os.sep) - base.count(os.sep) >= 2:
            dirs[:] = []
    return out


def main() -> int:
    res = {"self_nspid": [l for l in open("/proc/self/status").read().splitlines()
                          if l.startswith("NSpid")],
           "before": listing()}
    child = subprocess.Popen([sys.executable, "-c", CHILD], stdin=subprocess.PIPE,
                             stdout=subprocess.PIPE, text=True)
    line = child.stdout.readline().split()
    res["child_pid"] = int(line[0])
    res["child_nspid"] = line[1:]
    res["with_child"] = listing()
    new = [p for p in res["with_child"] if p not in res["before"]]
    res["new_entries"] = {p: entry(p) for p in new}
    res["new_entry_in_our_proc"] = {p: os.path.exists(f"/proc/{p}") for p in new}

    from gpumounter_amd.hw.inventory import Inventory
    from gpumounter_amd.node import procs
    inv = Inventory()
    gpus = inv.gpus()
    res["gpus"] = [{"index": g.index, "kfd_gpu_id": g.kfd_gpu_id, "render_minor": g.render_minor}
                   for g in gpus]
    res["after_smi_open"] = listing()
    res["amdsmi"] = {g.index: [vars(p) for p in inv.processes(g.index)] for g in gpus}
    hits, bad = procs.scan_devs([res["child_pid"]], [(226, g.render_minor) for g in gpus])
    res["fd_scan"] = {"hits": hits, "unreadable": bad}
    res["busy_auto"] = procs.busy_pids(inv, gpus, [res["child_pid"]])
    res["busy_both"] = procs.busy_pids(inv, gpus, [res["child_pid"]], mode="both")

    child.stdin.close()
    res["child_rc"] = child.wait(timeout=60)
    time.sleep(0.5)
    res["after_exit"] = listing()
    res["amdsmi_after_exit"] = {g.index: [p.pid for p in inv.processes(g.index)] for g in gpus}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/kfd_probe.json", "w") as fh:
        json.dump(res, fh, indent=1, default=str)
    print(json.dumps({k: res[k] for k in ("self_nspid", "child_pid", "child_nspid",
                                          "new_entry_in_our_proc", "amdsmi", "busy_auto",
                                          "busy_both")}, default=str))
    return 0


if __name__ == "__main__":
    sys.exit(main())
