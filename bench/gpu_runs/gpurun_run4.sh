set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
echo "== pytest gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r4/smoke.log; exit 1; }
cat gpurun_out/r4/smoke.log
echo "== bench default"
timeout -k 10 300 python bench.py > gpurun_out/r4/bench_default.json 2> gpurun_out/r4/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/r4/bench_default.err; exit 1; }
cut -c1-600 gpurun_out/r4/bench_default.json
echo "== bench 200 steps"
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > gpurun_out/r4/zero.json 2> gpurun_out/r4/zero.err || exit 1
cut -c1-400 gpurun_out/r4/zero.json
echo done
