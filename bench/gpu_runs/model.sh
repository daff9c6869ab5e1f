# Round 5 (profiles/r5_model/): the modes, the modelled real-cluster rows and the cold-path table.
#   gpurun --timeout 1100 -- bash bench/gpu_runs/model.sh <tag>
# 1. default / warm pool / DRA at zero latency (value, serial_calls_per_attach)
# 2. the same three with LatencyModel.realistic (api 1 ms, schedule 10, admit 15, ...): "modelled"
# 3. cold/first attach, interleaved: --deploy processes | inprocess × daemons pinned | not
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-model}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
run() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 300 python bench.py --gpus 1 "$@" > "$O/$name.json" 2>> "$O/bench.err" \
        || fail "$O/bench.err"
    python -c "import json; q=json.load(open('$O/$name.json')); a=q.get('serial_calls_per_attach') or {}; c=q.get('cold_attach') or {}; print('$name', q['value'], q['detach_p50_ms'], 'serial', a.get('serial_round_trips'), 'adm', a.get('admission_wait_p50_ms'), 'cold', q.get('cold_attach_p50_ms'), 'idle', (c.get('idle_only') or {}).get('attach_p50_ms'), 'first', q.get('first_attach_ms'))"
}
run zero_default --steps 20 --warmup 5 --cold-steps 0
run zero_pool --steps 20 --warmup 5 --cold-steps 0 --warm-pool 2
run zero_dra --steps 20 --warmup 5 --cold-steps 0 --gpu-api dra
run real_default --steps 10 --warmup 3 --cold-steps 0 --latency realistic --no-verify
run real_pool --steps 10 --warmup 3 --cold-steps 0 --latency realistic --warm-pool 2 --no-verify
run real_dra --steps 10 --warmup 3 --cold-steps 0 --latency realistic --gpu-api dra --no-verify
PIN=$(python -c "import os; c=sorted(os.sched_getaffinity(0)); print(f'{c[len(c)//2]}:{c[len(c)//2+1]}')")
echo "pinned daemons to $PIN"
for rep in 1 2; do
    run cold_proc_unpinned_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0
    run cold_proc_pinned_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0 --pin "$PIN"
    run cold_inproc_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0 --deploy inprocess
done
