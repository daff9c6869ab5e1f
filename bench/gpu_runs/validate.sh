# One-GPU MI355X validation pass, run from the repository root as
#   gpurun --timeout 1100 -- bash bench/gpu_runs/validate.sh <tag> [steps]
# Every GPU step has its own time limit; the first failing step ends the script.
# Results land in gpurun_out/<tag>/ and the ones worth keeping are copied into profiles/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
STEPS=${2:-100}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }

# 1-2: exactly what the driver runs at round end (from the repo root, no extra flags), each under
# a time limit of its own
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > "$O/pytest_gpu.log" 2>&1 || fail "$O/pytest_gpu.log"
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail "$O/smoke.log"
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/default.json" 2> "$O/default.err" || fail "$O/default.err"
timeout -k 10 300 python bench.py --gpus 1 --steps "$STEPS" --warmup 20 --warm-pool 1 \
    > "$O/pool.json" 2> "$O/pool.err" || fail "$O/pool.err"
timeout -k 10 300 python bench.py --gpus 1 --steps "$STEPS" --warmup 20 --gpu-api dra \
    > "$O/dra.json" 2> "$O/dra.err" || fail "$O/dra.err"
python - "$O" <<'PY'
import json, sys
for n in ("default", "pool", "dra"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    print(n, d["value"], d.get("attach_p99_ms"), d.get("detach_p50_ms"),
          d.get("ledger_audit_issues"), d.get("final_orphans"))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$O/rocprof" -o bench \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --deploy inprocess --steps 50 --warmup 10 --ref-steps 0 \
    > "$GRAFT_REPO_ROOT/$O/rocprof.log" 2>&1 || fail "$GRAFT_REPO_ROOT/$O/rocprof.log"
echo rocprof-ok
