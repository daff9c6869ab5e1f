# Round-6, second pass (after the cold phase sends the same master request in both kinds):
#   gpurun --timeout 1150 -- bash bench/gpu_runs/r6b.sh <tag>
# 1. the driver's command three times (attach p50; cold A/B interleaved on one master process);
# 2. 3000 timed cycles (the tail);
# 3. the modelled real cluster (LatencyModel.realistic): default, warm pool with standbys at the
#    floor class, warm pool with the low pool class (every attach yields the standby and books
#    the GPU at tenant rank: the price of preemptible standbys).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6b}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for i in 1 2 3; do
    timeout -k 10 300 python bench.py > "$O/default_$i.json" 2> "$O/default_$i.err" \
        || fail "$O/default_$i.err"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 3000 --warmup 50 --cold-steps 0 \
    --call-cycles 0 > "$O/soak3000.json" 2> "$O/soak3000.err" || fail "$O/soak3000.err"
for m in default pool_floor pool_low; do
    case $m in
        default) extra="" ;;
        pool_floor) extra="--warm-pool 1" ;;
        pool_low) extra="--warm-pool 1 --daemon-env GM_POOL_PRIORITY_CLASS=gpumounter-standby" ;;
    esac
    timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 --cold-steps 0 \
        --latency realistic --no-verify $extra > "$O/model_$m.json" 2> "$O/model_$m.err" \
        || fail "$O/model_$m.err"
done
python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("default_1", "default_2", "default_3", "soak3000", "model_default", "model_pool_floor",
          "model_pool_low"):
    d = json.load(open(f"{o}/{f}.json"))
    c = d.get("cold_attach") or {}
    print(f, d["value"], d["attach_p99_ms"], d.get("attach_p999_ms"), d["detach_p50_ms"],
          "cold", c.get("attach_p50_ms"), "idle", (c.get("idle_only") or {}).get("attach_p50_ms"),
          "authz", (c.get("stage_p50_ms") or {}).get("master_authz"),
          "first", d.get("first_attach_ms"))
PY
