# DRA-mode soak on one MI355X: bench.py --gpu-api dra (processes, mTLS + authz, real libamd_smi,
# liveness kernel after every attach), 3000 cycles with and without the warm pool: placeholders
# hold ResourceClaims; the ledger audit runs after every cycle.
#   gpurun --timeout 900 -- bash bench/gpu_runs/soak_dra.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-soak_dra}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --gpu-api dra \
    > "$O/dra_3000.json" 2> "$O/dra_3000.err" || fail "$O/dra_3000.err"
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --gpu-api dra --warm-pool 1 \
    > "$O/dra_pool_3000.json" 2> "$O/dra_pool_3000.err" || fail "$O/dra_pool_3000.err"
timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 20 --ref-steps 0 \
    > "$O/default_500.json" 2> "$O/default_500.err" || fail "$O/default_500.err"
python - "$O" <<'PY'
import json, sys
for f in ("dra_3000", "dra_pool_3000", "default_500"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, d["value"], d["attach_p99_ms"], d["attach_p999_ms"], d["attach_max_ms"],
          d["detach_p50_ms"], d["ledger_audit_issues"], d["final_orphans"], d["placeholders_left"])
PY
