# The CPU test suite (the driver's `pytest -m "not gpu"` gate) on a GPU box's CPU share:
#   gpurun --timeout 1150 -- bash bench/gpu_runs/cpu_suite.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-cpu_suite}
mkdir -p "$O"
timeout -k 10 1100 python -m pytest tests/ -x -q -m "not gpu" -n 12 --timeout 300 \
    > "$O/pytest.log" 2>&1
rc=$?
tail -15 "$O/pytest.log"
exit $rc
