set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r20
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || { tail -20 $O/default.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --warm-pool 1 > $O/pool.json 2> $O/pool.err || { tail -20 $O/pool.err; exit 1; }
python - <<'PY'
import json
for n in ("default","pool"):
    d=json.load(open(f"gpurun_out/r20/{n}.json")); print(n, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], d.get("reference_emulated_same_run"), d["ledger_audit_issues"], d["final_orphans"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r20/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench/gemm_sweep.py" --rounds 3 > "$GRAFT_REPO_ROOT/gpurun_out/r20/gemm_prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r20/gemm_prof.log"; exit 1; }
echo prof-ok
