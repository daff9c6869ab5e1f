# Block-scaled MFMA evidence on one MI355X: the GPU tests that cover it, the form sweep, the lane
# and scale maps, run-to-run determinism, and `probe --full` with the MX figures.
#   gpurun --timeout 900 -- bash bench/gpu_runs/mx_evidence.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-mx_evidence}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
timeout -k 10 300 python -m pytest tests/test_gpu.py -x -v -k "mx" --timeout 120 --timeout-method thread \
    > "$O/pytest_mx.log" 2>&1 || fail "$O/pytest_mx.log"
tail -5 "$O/pytest_mx.log"
timeout -k 10 200 python bench/mx_sweep.py > "$O/sweep.json" 2> "$O/sweep.err" || fail "$O/sweep.err"
timeout -k 10 120 python bench/mx_layout.py > "$O/layout.json" 2> "$O/layout.err" || fail "$O/layout.err"
timeout -k 10 120 python bench/mx_debug2.py > "$O/scale_lanes.json" 2> "$O/scale_lanes.err" || fail "$O/scale_lanes.err"
timeout -k 10 200 python bench/mx_det.py > "$O/determinism.json" 2> "$O/determinism.err" || fail "$O/determinism.err"
timeout -k 10 200 python -m gpumounter_amd probe --full > "$O/probe_full.json" 2> "$O/probe_full.err" || fail "$O/probe_full.err"
cat "$O/probe_full.json"
