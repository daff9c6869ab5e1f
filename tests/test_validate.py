"""Tenant-side validation tool (gpumounter_amd/parallel/validate.py): the all-reduce leg with
gloo ranks on the CPU; the GPU legs run in tests/test_gpu.py."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_validate_allreduce_over_cpu_ranks():
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": ""}
    res = subprocess.run([sys.executable, "-m", "gpumounter_amd.parallel.validate",
                          "--cpu-ranks", "2", "--numel", "4096"], cwd=ROOT, capture_output=True,
                         text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    rep = json.loads(res.stdout.strip().splitlines()[-1])
    assert rep["ok"] and rep["allreduce"]["world"] == 2 and rep["allreduce"]["ok"]
    assert rep["allreduce"]["bytes"] == 4096 * 4 and rep["allreduce"]["busbw_gbps"] > 0
