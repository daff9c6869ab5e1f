# The driver's command three times at the current tree (its spread on one box):
#   gpurun --timeout 600 -- bash bench/gpu_runs/driver3.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-driver3}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for i in 1 2 3; do
    timeout -k 10 300 python bench.py > "$O/default_$i.json" 2> "$O/default_$i.err" \
        || fail "$O/default_$i.err"
    python -c "import json; d=json.load(open('$O/default_$i.json')); print('default_$i', d['value'], d['attach_p99_ms'], d['detach_p50_ms'], d['attach_split_p50_ms'], d['box'].get('loadavg_1m'))"
done
