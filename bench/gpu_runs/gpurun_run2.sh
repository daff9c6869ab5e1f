set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu"
timeout -k 10 400 python -m pytest tests -m gpu -q -rA -s > gpurun_out/pytest_gpu2.log 2>&1; echo "pytest rc=$?"
grep -E "PASSED|FAILED|SKIPPED|passed|failed|amdsmi process|HBM" gpurun_out/pytest_gpu2.log | tail -25
echo "== bench zero-latency"
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench2.json 2> gpurun_out/bench2.err; echo "bench rc=$?"; cat gpurun_out/bench2.json
echo "== bench single-mount v1"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --mode single --cgroup v1 > gpurun_out/bench2_single_v1.json 2>> gpurun_out/bench2.err; echo "rc=$?"; cat gpurun_out/bench2_single_v1.json
echo "== bench realistic control plane"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --latency realistic > gpurun_out/bench2_realistic.json 2>> gpurun_out/bench2.err; echo "rc=$?"; cat gpurun_out/bench2_realistic.json
echo "== rocprofv3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d "$R/gpurun_out/prof2" -o bench --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$R/gpurun_out/prof2.log" 2>&1; echo "rocprof rc=$?"
tail -3 "$R/gpurun_out/prof2.log"
find "$R/gpurun_out/prof2" -name "*.csv" | head -20
