"""bench.py contract on CPU: single process and a 2-rank torch.distributed (gloo) launch, with the
mock inventory. The GPU box runs the same script with the real libamd_smi + HIP verification."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_single_process_json_line():
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    res = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "1",
                          "--amdsmi", "mock"], cwd=ROOT, capture_output=True, text=True,
                         timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _last_json(res.stdout)
    assert KEYS <= set(d)
    assert d["metric"] == "p50_gpu_attach_latency_ms" and d["higher_is_better"] is False
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["value"] > 0
    assert d["ledger_audit_issues"] == 0 and d["final_orphans"] == 0
    assert d["placeholders_left"] == 0


def test_bench_with_daemons_as_separate_processes():
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    res = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "1",
                          "--amdsmi", "mock", "--deploy", "processes"], cwd=ROOT,
                         capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _last_json(res.stdout)
    assert d["config"]["deploy"] == "processes" and d["value"] > 0
    assert d["ledger_audit_issues"] == 0 and d["final_orphans"] == 0
    assert d["placeholders_left"] == 0
    assert "daemon exit codes" not in res.stderr


def test_bench_dra_cluster_daemons():
    """--gpu-api dra: the daemons run with gpu_allocation=dra against the fake apiserver's
    resource.k8s.io/v1 (placeholders hold ResourceClaims)."""
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    res = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "1",
                          "--amdsmi", "mock", "--deploy", "processes", "--gpu-api", "dra"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _last_json(res.stdout)
    assert d["config"]["gpu_allocation"] == "dra" and d["value"] > 0
    assert d["ledger_audit_issues"] == 0 and d["final_orphans"] == 0
    assert d["placeholders_left"] == 0


def test_bench_two_rank_distributed_launch():
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--steps", "4", "--warmup", "1", "--amdsmi", "mock"]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _last_json(res.stdout)
    assert d["n_gpus"] == 2 and d["config"]["gpus_per_pod"] == 2
    assert d["ledger_audit_issues"] == 0


def test_baseline_config_scenarios_run_and_hold_invariants():
    """bench/configs.py: the BASELINE.json scenarios (short runs) report consistent ledgers."""
    import json as _json
    import subprocess as _sp
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for sc, extra in (("scale", []), ("contention", ["--rounds", "8"]),
                      ("soak", ["--cycles", "40"])):
        r = _sp.run([_sys.executable, os.path.join(root, "bench", "configs.py"), sc] + extra,
                    capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[sc] = _json.loads(r.stdout.strip().splitlines()[-1])
    assert out["scale"]["numa_packed"] and out["scale"]["audit_issues"] == 0
    assert [s["gpus"] for s in out["scale"]["steps"]] == list(range(1, 9))
    assert out["contention"]["invariant_violations"] == 0
    assert out["soak"]["orphaned_cgroup_entries"] == 0 == out["soak"]["orphaned_device_nodes"]
    assert out["soak"]["placeholders_left"] == 0 == out["soak"]["gpus_still_allocated"]


def test_bench_single_process_eight_gpus_verifies_every_per_n_field():
    """`bench.py --gpus 8` without a launcher (what a driver may run): all 8 attached, a collective
    over 8 spawned rank processes (gloo here, RCCL on MI355X), one hive, no non-xGMI pair."""
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "3", "--warmup",
                          "1", "--amdsmi", "mock", "--deploy", "inprocess", "--ref-steps", "0"],
                         cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _last_json(res.stdout)
    assert d["n_gpus"] == 8 and d["config"]["gpus_per_pod"] == 8
    if os.path.isdir("/sys/class/kfd/kfd/topology/nodes"):
        # a GPU box: the mock inventory's GPUs are not the box's, so bench.py measures the
        # control plane alone and runs no collective over them
        assert d["allreduce_backend"] is None
    else:
        assert d["allreduce_backend"] == "gloo" and d["allreduce_2MiB_p50_ms"] > 0
    assert d["rccl_allreduce_2MiB_p50_ms"] is None          # no RCCL claim without a GPU
    assert d["attached_hives"] == 1 and d["non_xgmi_pairs"] == 0
    assert d["node_ops"] == "emulated" and d["dtype"] == "none"
    assert d["ledger_audit_issues"] == 0 and d["final_orphans"] == 0
    assert d["placeholders_left"] == 0


def test_bench_real_node_ops_reports_stage_split():
    from gpumounter_amd.fakes import realnode
    import pytest
    from conftest import privileged_ok
    if realnode.available() or not privileged_ok():
        pytest.skip("needs root with mount + bpf (mounts cgroup2/bpffs)")
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    # --ref-steps with real node ops: the reference column is skipped with its reason, never
    # a crash
    res = subprocess.run([sys.executable, "bench.py", "--steps", "10", "--warmup", "2",
                          "--amdsmi", "mock", "--node-ops", "real", "--ref-steps", "5"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _last_json(res.stdout)
    assert d["node_ops"] == "real" and d["attach_p50_real_node_ops_ms"] == d["value"]
    st = d["real_node_ops_stage_p50_ms"]
    assert {"bpf_load_verify", "bpf_attach", "devnodes", "cgroup_rule"} <= set(st)
    assert d["ledger_audit_issues"] == 0 and d["final_orphans"] == 0
    assert "cgroup-v1" in d["reference_emulated_same_run"]["skipped"]


def test_rank_pool_two_ranks_on_cpu():
    """bench.py --gpus N without a launcher: the spawned rank processes rendezvous through a
    file (no pre-picked TCP port) and all-reduce; gloo on the CPU here, RCCL on a GPU node."""
    code = ("import json; from gpumounter_amd.parallel.rankpool import RankPool; "
            "p = RankPool(2); r = p.allreduce(['0000:15:00.0', '0000:05:00.0'], 1024); "
            "r2 = p.allreduce(['0000:15:00.0', '0000:05:00.0'], 1024); "
            "print(json.dumps([r, r2, p.close()]))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=180, cwd=ROOT, env={**os.environ, "CUDA_VISIBLE_DEVICES": "",
                                                     "GM_RANKPOOL_CPU": "1"})
    assert out.returncode == 0, out.stderr[-3000:]
    r, r2, codes = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["ok"] and r2["ok"] and r["backend"] == "gloo"
    assert r["bdfs"] == ["0000:05:00.0", "0000:15:00.0"]      # rank r ↔ sorted(bdfs)[r]
    assert codes == {"0": 0, "1": 0}
