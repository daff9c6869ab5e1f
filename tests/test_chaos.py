"""bench/configs.py chaos, short: four Pods attaching and detaching over HTTP against the process
deployment while the worker injects faults at every mutating stage and is SIGKILLed twice with
requests in flight, 5 % of the apiserver's Pod requests fail (some after taking effect) and
tenant containers restart mid-request.
The ledger invariants hold after every round (see chaos() for the list). Variants: every GPU
busy with a SIGTERM-ignoring process (force removals), and attaches with short leases."""
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


def test_chaos_with_busy_gpus_kills_before_releasing():
    """--busy: every hot-mounted GPU is used by a SIGTERM-ignoring process of its tenant, so each
    removal is a force removal that must kill it first; one worker SIGKILL lands mid-drain at
    some point. No GPU is released while its process runs, and every success names only
    processes that are gone."""
    res = subprocess.run([sys.executable, "bench/configs.py", "chaos", "--busy", "--rounds", "10",
                          "--kill-every", "5", "--seed", "2", "--busy-pool", "12"], cwd=ROOT,
                         capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["worker_kills"] == 2 and out["busy"]["force_kills_answered"] > 0
    assert out["busy"]["processes_killed"] >= out["busy"]["force_kills_answered"]
    assert out["invariant_violations"] == 0, out["violation_examples"]


def test_chaos_with_leases_ends_them_across_worker_kills():
    """--lease-rate: half the attaches carry a 0.1-0.5 s lease (?lease=). With the worker
    SIGKILLed twice, every lease has ended within --lease-slack of its expiry and unleased GPUs
    stay exactly as their client left them."""
    res = subprocess.run([sys.executable, "bench/configs.py", "chaos", "--lease-rate", "0.5",
                          "--rounds", "12", "--kill-every", "6", "--seed", "3"], cwd=ROOT,
                         capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["worker_kills"] == 2 and out["leases"]["attached"] > 0
    assert out["invariant_violations"] == 0, out["violation_examples"]


def test_chaos_with_preemptors_never_takes_a_tenants_gpu():
    """--preempt-rate: a priority-1000 Pod that wants every GPU of node-0 comes and goes while
    the worker is SIGKILLed. Under the shipped floor class no placeholder that books a tenant's
    GPU is ever its victim — only idle standbys at the low pool class are. The negative control,
    placeholders at the reference's priority 0, has the scheduler preempt them."""
    base = [sys.executable, "bench/configs.py", "chaos", "--rounds", "8", "--kill-every", "4",
            "--seed", "5", "--restart-rate", "0.3", "--preempt-rate", "1", "--preempt-gpus", "8"]
    res = subprocess.run(base + ["--warm-pool", "2", "--pool-priority-class",
                                 "gpumounter-standby"], cwd=ROOT, capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["preemptors"] > 0 and out["preempted"]["placeholder"] == 0
    assert out["invariant_violations"] == 0, out["violation_examples"]
    res = subprocess.run(base + ["--no-placeholder-priority"], cwd=ROOT, capture_output=True,
                         text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["preempted"]["placeholder"] > 0
    assert any("preempted" in v for v in out["violation_examples"]), out["violation_examples"]


def test_chaos_with_a_kubelet_that_tears_down_late_and_keeps_deleted_pods_checkpointed():
    """--latency teardown --lazy-checkpoint: the fake kubelet frees a deleted Pod's devices
    50 ms after the DELETE and keeps it in its device-manager checkpoint until the next
    Allocate, as a real kubelet does. Attaches and pool refills right after a detach are
    refused at admission and book again; the ledger invariants hold across worker kills."""
    res = subprocess.run([sys.executable, "bench/configs.py", "chaos", "--rounds", "10",
                          "--kill-every", "5", "--seed", "6", "--restart-rate", "0.3",
                          "--latency", "teardown", "--lazy-checkpoint", "--warm-pool", "2",
                          "--placeholder-binding", "direct"], cwd=ROOT, capture_output=True,
                         text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["worker_kills"] == 2 and out["ops_ok"] > 0
    assert out["invariant_violations"] == 0, out["violation_examples"]
