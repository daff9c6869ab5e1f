set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
echo "== pytest gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" $O/pytest_gpu.log | tail -25
if [ $rc -ge 124 ] || [ $rc -eq 134 ]; then echo "pytest crashed: stop"; exit 1; fi
grep -B5 -A30 "amd_smi_tool_sees" $O/pytest_gpu.log | grep -E "Error|assert|found" | head -10
echo "== amd-smi list"
timeout -k 5 60 amd-smi list --json > $O/amd_smi_list.json 2>&1; head -c 1200 $O/amd_smi_list.json; echo
echo "== bench default"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
echo "== bench zero 200"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/zero.json 2> $O/zero.err || exit 1
echo "== bench pool 200"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --warm-pool 1 > $O/pool.json 2> $O/pool.err || exit 1
echo "== bench realistic"
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --latency realistic > $O/realistic.json 2> $O/realistic.err || exit 1
python - <<'PY'
import json
for n in ("zero","pool","realistic"):
    d=json.load(open(f"gpurun_out/r5/{n}.json")); print(n, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], d.get("reference_emulated_same_run"))
PY
echo "== rocprofv3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d "$R/$O/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 5 > "$R/$O/prof.log" 2>&1; echo "rocprof rc=$?"
find "$R/$O/prof" -name "*stats.csv" | head
echo done
