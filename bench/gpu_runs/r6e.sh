# Round-6, fifth pass: the modelled real cluster (LatencyModel.realistic, now with a 50 ms kubelet
# teardown of deleted Pods) for every placeholder binding × warm-pool class, on the box's one
# GPU (each attach books the GPU the previous detach freed) and on the mock 8-GPU inventory:
#   gpurun --timeout 900 -- bash bench/gpu_runs/r6e.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6e}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
LOW="--daemon-env GM_POOL_PRIORITY_CLASS=gpumounter-standby"
DIRECT="--daemon-env GM_PLACEHOLDER_BINDING=direct"
for m in scheduler direct pool_floor pool_floor_direct pool_low pool_low_direct \
         mock8_scheduler mock8_direct mock8_pool_low; do
    case $m in
        scheduler) extra="" ;;
        direct) extra="$DIRECT" ;;
        pool_floor) extra="--warm-pool 1" ;;
        pool_floor_direct) extra="--warm-pool 1 $DIRECT" ;;
        pool_low) extra="--warm-pool 1 $LOW" ;;
        pool_low_direct) extra="--warm-pool 1 $LOW $DIRECT" ;;
        # the mock 8-GPU inventory: the GPU an attach books is never the one just detached,
        # so the kubelet's teardown is off the attach path
        mock8_scheduler) extra="--amdsmi mock" ;;
        mock8_direct) extra="--amdsmi mock $DIRECT" ;;
        mock8_pool_low) extra="--amdsmi mock --warm-pool 1 $LOW" ;;
    esac
    timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 3 --cold-steps 0 \
        --latency realistic --no-verify $extra > "$O/model_$m.json" 2> "$O/model_$m.err" \
        || fail "$O/model_$m.err"
done
python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("scheduler", "direct", "pool_floor", "pool_floor_direct", "pool_low", "pool_low_direct",
          "mock8_scheduler", "mock8_direct", "mock8_pool_low"):
    d = json.load(open(f"{o}/model_{f}.json"))
    st = d.get("stage_p50_ms") or {}
    print(f, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], "wait",
          st.get("placeholder_wait"), "reserve", st.get("ledger_reserve"),
          "calls", (d.get("serial_calls_per_attach") or {}).get("by_process", {}).get("worker"))
PY
