set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" $O/pytest_gpu.log | tail -20
if [ $rc -ne 0 ]; then tail -40 $O/pytest_gpu.log; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > $O/zero.json 2> $O/zero.err || { tail -20 $O/zero.err; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --warm-pool 1 > $O/pool.json 2> $O/pool.err || { tail -20 $O/pool.err; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --latency realistic > $O/realistic.json 2> $O/realistic.err || { tail -20 $O/realistic.err; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --latency realistic --protocol reference > $O/ref_realistic.json 2> $O/ref_realistic.err || { tail -20 $O/ref_realistic.err; exit 1; }
python - <<'PY'
import json
for n in ("bench_default","zero","pool","realistic","ref_realistic"):
    d=json.load(open(f"gpurun_out/r9/{n}.json")); print(n, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], d["config"]["deploy"], d.get("reference_emulated_same_run"))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d "$R/$O/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 10 --ref-steps 0 > "$R/$O/prof.log" 2>&1; echo "rocprof rc=$?"
find "$R/$O/prof" -name "*stats.csv" | head -20
