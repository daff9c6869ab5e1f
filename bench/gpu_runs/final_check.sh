# The driver's command and one modelled run on the box's one GPU, at the current tree:
#   gpurun --timeout 600 -- bash bench/gpu_runs/final_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-final_check}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
timeout -k 10 300 python bench.py > "$O/default.json" 2> "$O/default.err" || fail "$O/default.err"
timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 3 --cold-steps 0 \
    --latency realistic --no-verify > "$O/model.json" 2> "$O/model.err" || fail "$O/model.err"
for f in default model; do
    python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['attach_p99_ms'], d.get('admission_refusals'), d.get('final_orphans'))"
done
