# MX-MFMA numerics localisation (bench/mx_debug.py) on one MI355X.
#   gpurun --timeout 300 -- bash bench/gpu_runs/mx_debug.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-mx_debug}
mkdir -p "$O"
timeout -k 10 120 python bench/mx_sweep.py > "$O/debug.json" 2> "$O/debug.err" || { tail -40 "$O/debug.err"; exit 1; }
cat "$O/debug.json"
