# BASELINE.json's named configurations on one MI355X box (bench/configs.py), run from the
# repository root as
#   gpurun --timeout 900 -- bash bench/gpu_runs/configs.sh <tag>
# scale / contention / soak on the bundled 8×MI355X mock inventory (the box has one GPU), then the
# 1000-cycle soak on the real libamd_smi inventory, then the contention scenario with every
# daemon in its own process (clients over HTTP). Each step has its own time limit; the first
# failing step ends the script. Results land in gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-configs}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for s in scale contention soak placement; do
    timeout -k 10 240 python bench/configs.py "$s" > "$O/${s}_mock.json" 2> "$O/${s}_mock.err" \
        || fail "$O/${s}_mock.err"
    tail -c 400 "$O/${s}_mock.json"; echo
done
timeout -k 10 240 python bench/configs.py soak --amdsmi "" > "$O/soak_real.json" 2> "$O/soak_real.err" \
    || fail "$O/soak_real.err"
tail -c 400 "$O/soak_real.json"; echo
timeout -k 10 240 python bench/configs.py contention --deploy processes \
    > "$O/contention_processes.json" 2> "$O/contention_processes.err" \
    || fail "$O/contention_processes.err"
tail -c 400 "$O/contention_processes.json"; echo
