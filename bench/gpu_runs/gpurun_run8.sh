set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r8
mkdir -p $O
timeout -k 10 400 python bench/configs.py soak --amdsmi "" > $O/soak_real.json 2> $O/soak_real.err || { tail -20 $O/soak_real.err; exit 1; }
echo "soak real: $(cut -c1-400 $O/soak_real.json)"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --deploy processes > $O/zero_processes.json 2> $O/zero_processes.err || { tail -20 $O/zero_processes.err; exit 1; }
echo "processes: $(cut -c1-200 $O/zero_processes.json)"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/zero.json 2> $O/zero.err || { tail -20 $O/zero.err; exit 1; }
python - <<'PY'
import json
for n in ("zero","zero_processes"):
    d=json.load(open(f"gpurun_out/r8/{n}.json")); print(n, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], d["stage_p50_ms"], d.get("reference_emulated_same_run"))
PY
