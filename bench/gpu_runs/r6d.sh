# Round-6, fourth pass: placeholder binding on the modelled real cluster (LatencyModel.realistic).
#   gpurun --timeout 900 -- bash bench/gpu_runs/r6d.sh <tag>
# scheduler (the default: kube-scheduler binds each placeholder) vs direct (spec.nodeName at
# creation, no scheduling cycle), each without and with a warm pool; then the driver's command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6d}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for m in scheduler direct scheduler_pool direct_pool; do
    case $m in
        scheduler) extra="" ;;
        direct) extra="--daemon-env GM_PLACEHOLDER_BINDING=direct" ;;
        scheduler_pool) extra="--warm-pool 1" ;;
        direct_pool) extra="--warm-pool 1 --daemon-env GM_PLACEHOLDER_BINDING=direct" ;;
    esac
    timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 3 --cold-steps 0 \
        --latency realistic --no-verify $extra > "$O/model_$m.json" 2> "$O/model_$m.err" \
        || fail "$O/model_$m.err"
done
timeout -k 10 300 python bench.py > "$O/default.json" 2> "$O/default.err" || fail "$O/default.err"
python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("model_scheduler", "model_direct", "model_scheduler_pool", "model_direct_pool",
          "default"):
    d = json.load(open(f"{o}/{f}.json"))
    st = d.get("stage_p50_ms") or {}
    print(f, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], "wait",
          st.get("placeholder_wait"), "reserve", st.get("ledger_reserve"),
          "first", d.get("first_attach_ms"))
PY
