# 1/2/4/8 GPUs per attach on the mock 8-GPU inventory, and the warm pool with both standby
# classes, at the current tree:
#   gpurun --timeout 900 -- bash bench/gpu_runs/scale_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-scale_final}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for n in 1 2 4 8; do
    timeout -k 10 240 python bench.py --amdsmi mock --gpus $n --steps 100 --warmup 20 \
        --cold-steps 0 > "$O/mock_n$n.json" 2> "$O/mock_n$n.err" || fail "$O/mock_n$n.err"
    python -c "import json; d=json.load(open('$O/mock_n$n.json')); print('mock_n$n', d['value'], d['attach_p99_ms'], d['detach_p50_ms'])"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --warm-pool 1 \
    --daemon-env GM_POOL_PRIORITY_CLASS=gpumounter-standby \
    > "$O/pool_low.json" 2> "$O/pool_low.err" || fail "$O/pool_low.err"
python -c "import json; d=json.load(open('$O/pool_low.json')); print('pool_low', d['value'], d['attach_p99_ms'], d.get('admission_refusals'))"
