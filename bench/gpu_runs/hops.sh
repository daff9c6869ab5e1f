# Where the attach time outside the worker goes, on one box:
#   gpurun --timeout 900 -- bash bench/gpu_runs/hops.sh <tag>
# the driver's bench command three times (JSON: box calibration incl. the gRPC floor, master
# stages gm:master_*, worker rpc_queue/rpc_tail), then the gRPC transport floor with a handler
# that answers at once / awaits / makes HTTP calls. Results: gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-hops}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
for i in 1 2 3; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
        --dump-samples "$O/b$i.samples.jsonl" > "$O/b$i.json" 2> "$O/b$i.err" || { tail -30 "$O/b$i.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['attach_split_p50_ms'], d['master_stage_p50_ms'], {k: v for k, v in d['stage_p50_ms'].items() if k.startswith('rpc')}, d['box'])" "$O/b$i.json"
done
for r in 1 2; do
    for m in idle sleep http "idle lat" "http lat"; do
        timeout -k 10 120 python3 bench/gpu_runs/hop_floor.py $m | tee -a "$O/floor.txt" || exit 1
    done
done
