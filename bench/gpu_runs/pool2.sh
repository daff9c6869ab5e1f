# The warm-pool bench twice and the driver's command once more, at the current tree:
#   gpurun --timeout 600 -- bash bench/gpu_runs/pool2.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pool2}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for i in 1 2; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --warm-pool 1 \
        > "$O/pool_$i.json" 2> "$O/pool_$i.err" || fail "$O/pool_$i.err"
    python -c "import json; d=json.load(open('$O/pool_$i.json')); print('pool_$i', d['value'], d['attach_p99_ms'], d['probe_quick_p50_us'])"
done
timeout -k 10 300 python bench.py > "$O/default.json" 2> "$O/default.err" || fail "$O/default.err"
python -c "import json; d=json.load(open('$O/default.json')); print('default', d['value'], d['attach_p99_ms'], d['probe_quick_p50_us'])"
