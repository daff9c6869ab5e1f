# Round-6, the low pool class after cancel_pending_low (an attach cancels low standbys still
# being admitted): zero-latency and modelled, next to the floor-class pool.
#   gpurun --timeout 900 -- bash bench/gpu_runs/r6c.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6c}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
LOW="--daemon-env GM_POOL_PRIORITY_CLASS=gpumounter-standby"
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --warm-pool 1 --cold-steps 0 \
    > "$O/pool_floor.json" 2> "$O/pool_floor.err" || fail "$O/pool_floor.err"
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --warm-pool 1 --cold-steps 0 \
    $LOW > "$O/pool_low.json" 2> "$O/pool_low.err" || fail "$O/pool_low.err"
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 --cold-steps 0 \
    --latency realistic --no-verify --warm-pool 1 $LOW > "$O/model_pool_low.json" \
    2> "$O/model_pool_low.err" || fail "$O/model_pool_low.err"
python - "$O" <<'PY'
import json, sys
for f in ("pool_floor", "pool_low", "model_pool_low"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    a = d.get("serial_calls_per_attach") or {}
    print(f, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], "serial",
          a.get("serial_round_trips"), {k: v for k, v in d["stage_p50_ms"].items() if v > 0.1})
PY
