set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
B="timeout -k 10 400 python bench.py"
run() { name=$1; shift; $B "$@" > gpurun_out/r3/$name.json 2> gpurun_out/r3/$name.err; rc=$?; echo "$name rc=$rc"; cut -c1-400 gpurun_out/r3/$name.json; return $rc; }
echo "== pytest gpu"
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/r3/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r3/pytest_gpu.log
run ours_zero --steps 200 --warmup 20 &&
run ours_zero_pool --steps 200 --warmup 20 --warm-pool 1 &&
run ref_zero --steps 50 --warmup 5 --protocol reference &&
run ours_real --steps 20 --warmup 2 --latency realistic &&
run ours_real_pool --steps 20 --warmup 2 --latency realistic --warm-pool 1 &&
run ref_real --steps 3 --warmup 1 --latency realistic --protocol reference
echo done
