set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r15
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
grep -E "ECC|passed|failed" $O/pytest_gpu.log | tail -5
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || { tail -20 $O/default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --latency realistic > $O/realistic.json 2> $O/realistic.err || { tail -20 $O/realistic.err; exit 1; }
timeout -k 10 400 python bench/configs.py soak --amdsmi "" --cycles 3000 > $O/soak_real_3000.json 2> $O/soak.err || { tail -20 $O/soak.err; exit 1; }
python - <<'PY'
import json
for n in ("default","realistic"):
    d=json.load(open(f"gpurun_out/r15/{n}.json")); print(n, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], d["stage_p50_ms"].get("placeholder_wait"), d.get("reference_emulated_same_run"))
print(open("gpurun_out/r15/soak_real_3000.json").read()[:400])
PY
