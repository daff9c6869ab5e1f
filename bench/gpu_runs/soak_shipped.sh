# Tail latency of the shipped deployment shape on one MI355X: bench.py (processes, mTLS + authz,
# real libamd_smi, gfx950 liveness kernel after every attach) for 3000 timed cycles, with and
# without the warm pool. p50/p99/p99.9/max and the ledger audit after every cycle.
#   gpurun --timeout 900 -- bash bench/gpu_runs/soak_shipped.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-soak_shipped}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --ref-steps 0 \
    > "$O/default_3000.json" 2> "$O/default_3000.err" || fail "$O/default_3000.err"
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --warm-pool 1 \
    > "$O/pool_3000.json" 2> "$O/pool_3000.err" || fail "$O/pool_3000.err"
python - "$O" <<'PY'
import json, sys
for f in ("default_3000", "pool_3000"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, d["value"], d["attach_p99_ms"], d["attach_p999_ms"], d["attach_max_ms"],
          d["detach_p50_ms"], d["ledger_audit_issues"], d["final_orphans"], d["placeholders_left"])
PY
