# Attach latency of the other shipped modes on one MI355X box (the headline is the default mode):
#   gpurun --timeout 900 -- bash bench/gpu_runs/modes.sh <tag>
# warm pool (claim instead of create), DRA placeholders, trim placement, own device plugin (the
# fake kubelet drives the plugin in-process, so that run is --deploy inprocess).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-modes}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
run() {
    name=$1; shift
    timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --cold-steps 0 "$@" \
        > "$O/$name.json" 2> "$O/$name.err" || { tail -20 "$O/$name.err"; exit 1; }
    python - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["value"], d["attach_p99_ms"], "detach", d["detach_p50_ms"],
      {k: v for k, v in d["stage_p50_ms"].items() if v >= 0.05 and "." not in k})
PY
}
run default
run pool --warm-pool 2
run dra --gpu-api dra
run trim --placement trim
run plugin --device-plugin --deploy inprocess
