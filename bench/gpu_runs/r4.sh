# Round-4 validation pass on one MI355X, from the repository root:
#   gpurun --timeout 1100 -- bash bench/gpu_runs/r4.sh <tag>
# 1. the driver's GPU gate (pytest -m gpu) and smoke()
# 2. the driver's bench command three times (box calibration, master stages, cold attach)
# 3. the gRPC hop in isolation (bench/gpu_runs/hop_floor.py), shipped options added one by one
# 4. 3000 timed cycles with every sample dumped, and the tail attribution (bench/tail_report.py)
# 5. rocprofv3 kernel + marker trace of the in-process deployment (gm:* and gm:master_* ranges)
# Every GPU step has its own time limit; the first failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }

timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1 || fail "$O/pytest_gpu.log"
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || fail "$O/smoke.log"
tail -1 "$O/smoke.log"
for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
        --dump-samples "$O/bench$i.jsonl" > "$O/bench$i.json" 2> "$O/bench$i.err" || fail "$O/bench$i.err"
    python - "$O/bench$i.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("bench", d["value"], d["attach_p99_ms"], d["attach_split_p50_ms"], "cold",
      d["cold_attach_p50_ms"], (d["cold_attach"] or {}).get("idle_only", {}).get("attach_p50_ms"),
      "first", d["first_attach_ms"], "probe", d["probe_quick_p50_us"])
PY
done
for o in "" "--http" "--http --shield" "--http --big" "--http --retry" "--http --tls" \
         "--http --tls --retry --big --shield"; do
    timeout -k 10 120 python bench/gpu_runs/hop_floor.py $o | tee -a "$O/hop_floor.jsonl" || exit 1
done
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --cold-steps 0 \
    --dump-samples "$O/soak.jsonl" > "$O/soak.json" 2> "$O/soak.err" || fail "$O/soak.err"
python bench/tail_report.py "$O/soak.jsonl" > "$O/tail_report.json"
python - "$O/tail_report.json" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))[0]
print("soak", r["attach_ms"], "tail excess", dict(list(r["tail_excess_over_p50_ms"].items())[:5]))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -f csv -d "$O/rocprof" -o bench \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --deploy inprocess --steps 50 --warmup 10 --cold-steps 0 \
    > "$O/rocprof.log" 2>&1 || fail "$O/rocprof.log"
echo rocprof-ok
