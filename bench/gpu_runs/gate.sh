# The driver's round-end GPU gate and nothing else: `pytest -m gpu` then smoke(), as the driver
# runs them, plus the list of in-tree shared objects those processes mapped.
#   gpurun --timeout 900 -- bash bench/gpu_runs/gate.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-gate}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
GM_RECORD_MAPS="$O/maps_pytest.txt" timeout -k 10 600 python -m pytest tests/ -x -q -m gpu \
    > "$O/pytest_gpu.log" 2>&1 || fail "$O/pytest_gpu.log"
tail -3 "$O/pytest_gpu.log"
GM_RECORD_MAPS="$O/maps_smoke.txt" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
    > "$O/smoke.log" 2>&1 || fail "$O/smoke.log"
tail -1 "$O/smoke.log"
cat "$O"/maps_*.txt 2>/dev/null
