# Long attach/detach soak for the tail (p99.9) of the driver's command, no profiler attached:
#   gpurun --timeout 900 -- bash bench/gpu_runs/soak_long.sh <tag> [cycles]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-soak_long}
N=${2:-30000}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for i in 1 2; do
    timeout -k 10 400 python bench.py --gpus 1 --steps "$N" --warmup 100 --cold-steps 0 \
        --dump-samples "$O/soak$i.jsonl" > "$O/soak$i.json" 2>> "$O/bench.err" || fail "$O/bench.err"
    python bench/tail_report.py "$O/soak$i.jsonl" > "$O/tail_report$i.json" || true
    gzip -f "$O/soak$i.jsonl"
    python -c "import json; q=json.load(open('$O/soak$i.json')); print('soak', q['value'], q['attach_p99_ms'], q.get('attach_p999_ms'), q['attach_split_p50_ms'], q['detach_p50_ms'])"
done
