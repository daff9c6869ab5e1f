# The gRPC hop split into its request and response legs (master send → worker handler, handler
# return → master receive; same-host monotonic clock), with and without what else runs on the
# worker's loop:
#   gpurun --timeout 900 -- bash bench/gpu_runs/legs.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-legs}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
run() {   # name, extra env assignments...
    n=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --cold-steps 0 \
        --no-calib --dump-samples "$O/$n.jsonl" > "$O/$n.json" 2> "$O/$n.err" || { tail -30 "$O/$n.err"; exit 1; }
    python3 - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
m = d["master_stage_p50_ms"]
print(sys.argv[2], d["value"], d["attach_split_p50_ms"], "req", m.get("master_rpc.grpc_request"),
      "resp", m.get("master_rpc.grpc_response"),
      {k: v for k, v in d["stage_p50_ms"].items() if k.startswith("rpc_")})
PY
}
run base GM_X=0
run no_events GM_EMIT_EVENTS=false
run no_guard GM_DEVICE_GUARD_PERIOD_S=0
run base2 GM_X=0
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --cold-steps 0 --no-calib \
    --security off > "$O/insecure.json" 2> "$O/insecure.err" || { tail -30 "$O/insecure.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); m=d['master_stage_p50_ms']; print('insecure', d['value'], d['attach_split_p50_ms'], m.get('master_rpc.grpc_request'), m.get('master_rpc.grpc_response'))" "$O/insecure.json"
