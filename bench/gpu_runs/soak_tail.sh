# Tail-latency attribution on one MI355X: 3000 attach/detach cycles of the shipped shape, device
# plugin and DRA, every timed attach dumped with the worker's stage split (bench.py
# --dump-samples); the summary names where the slowest cycles spent their time.
#   gpurun --timeout 900 -- bash bench/gpu_runs/soak_tail.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-soak_tail}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
mkdir -p "$O/logs_default"
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --ref-steps 0 \
    --log-dir "$O/logs_default" --dump-samples "$O/default.jsonl" > "$O/default.json" 2> "$O/default.err" || fail "$O/default.err"
mkdir -p "$O/logs_dra"
timeout -k 10 400 python bench.py --gpus 1 --steps 3000 --warmup 50 --gpu-api dra \
    --log-dir "$O/logs_dra" --dump-samples "$O/dra.jsonl" > "$O/dra.json" 2> "$O/dra.err" || fail "$O/dra.err"
python bench/tail_report.py "$O/default.jsonl" "$O/dra.jsonl" > "$O/tail_report.json"
cat "$O/tail_report.json"
