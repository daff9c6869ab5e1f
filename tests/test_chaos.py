"""bench/configs.py chaos, short: four Pods attaching and detaching over HTTP against the process
deployment while the worker injects faults at every mutating stage and is SIGKILLed twice with
requests in flight, 5 % of the apiserver's Pod requests fail (some after taking effect) and
tenant containers restart mid-request.
The ledger invariants hold after every round (see chaos() for the list)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chaos_keeps_the_ledger_invariants():
    res = subprocess.run([sys.executable, "bench/configs.py", "chaos", "--rounds", "8",
                          "--kill-every", "4", "--seed", "1", "--api-fault-rate", "0.05",
                          "--restart-rate", "0.5"], cwd=ROOT, capture_output=True,
                         text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["worker_kills"] == 2 and out["ops_ok"] > 0 and out["api_faults_served"] > 0
    assert out["invariant_violations"] == 0, out["violation_examples"]
