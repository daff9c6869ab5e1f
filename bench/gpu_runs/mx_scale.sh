# MX-MFMA scale coverage and determinism exploration (bench/mx_scale.py) on one MI355X.
#   gpurun --timeout 300 -- bash bench/gpu_runs/mx_scale.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-mx_scale}
mkdir -p "$O"
timeout -k 10 180 python bench/mx_scale.py > "$O/scale.json" 2> "$O/scale.err" || { tail -40 "$O/scale.err"; exit 1; }
cat "$O/scale.json"
timeout -k 10 120 python bench/mx_debug.py > "$O/debug.json" 2> "$O/debug.err" || { tail -40 "$O/debug.err"; exit 1; }
cat "$O/debug.json"
