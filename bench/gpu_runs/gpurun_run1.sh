set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== rocm-smi"; (rocm-smi --showbus --showproductname 2>&1 | head -30) || true
echo "== pytest gpu"
timeout -k 10 400 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -30 gpurun_out/pytest_gpu.log
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"
tail -5 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
