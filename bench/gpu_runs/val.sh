# GPU validation of the tree as it is: the gate, smoke, the driver's command three times with
# the first-attach split printed.
#   gpurun --timeout 900 -- bash bench/gpu_runs/val.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-val}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
GM_RECORD_MAPS="$O/maps_pytest.txt" timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu \
    --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || fail "$O/pytest_gpu.log"
tail -2 "$O/pytest_gpu.log"
GM_RECORD_MAPS="$O/maps_smoke.txt" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
    > "$O/smoke.log" 2>&1 || fail "$O/smoke.log"
tail -1 "$O/smoke.log"
for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench$i.json" \
        2>> "$O/bench.err" || fail "$O/bench.err"
    python - "$O/bench$i.json" <<'EOF'
import json, sys
q = json.load(open(sys.argv[1]))
f = q.get("first_attach_stages_ms") or {}
split = {"http+client": round(f["client"] - f["master"] - f.get("master.master_authz", 0), 3),
         "authz": f.get("master.master_authz"),
         "hop": round(f["master.master_rpc"] - f["worker"], 3), "worker": round(f["worker"], 3)}
print("bench", q["value"], q["attach_split_p50_ms"], "detach", q["detach_p50_ms"],
      "cold", q["cold_attach_p50_ms"], "first", q["first_attach_ms"], split)
EOF
done
