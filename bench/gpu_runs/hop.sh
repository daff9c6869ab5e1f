# Attribution of the client → master → worker hops (round 5, profiles/r5_hop/):
#   1. the GPU gate (pytest -m gpu, smoke) on the tree as it is;
#   2. the driver's command three times (value, attach_split_p50_ms, box floors);
#   3. 3000 cycles with both daemons under the stack sampler (GM_PROFILE_MODE=sample) and
#      every cycle dumped for bench/tail_report.py.
#   gpurun --timeout 1100 -- bash bench/gpu_runs/hop.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-hop}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
GM_RECORD_MAPS="$O/maps_pytest.txt" timeout -k 10 600 python -m pytest tests/ -x -q -m gpu \
    > "$O/pytest_gpu.log" 2>&1 || fail "$O/pytest_gpu.log"
tail -2 "$O/pytest_gpu.log"
GM_RECORD_MAPS="$O/maps_smoke.txt" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
    > "$O/smoke.log" 2>&1 || fail "$O/smoke.log"
tail -1 "$O/smoke.log"
for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench$i.json" \
        2>> "$O/bench.err" || fail "$O/bench.err"
    python -c "import json,sys; q=json.load(open('$O/bench$i.json')); print('bench', q['value'], q['attach_split_p50_ms'], q['detach_p50_ms'], q['cold_attach_p50_ms'], q['first_attach_ms'])"
done
mkdir -p "$O/prof"
GM_PROFILE_OUT="$PWD/$O/prof/{pid}.json" GM_PROFILE_MODE=sample timeout -k 10 600 \
    python bench.py --gpus 1 --steps 3000 --warmup 50 --cold-steps 0 \
    --dump-samples "$O/soak.jsonl" > "$O/soak.json" 2>> "$O/bench.err" || fail "$O/bench.err"
python bench/tail_report.py "$O/soak.jsonl" > "$O/tail_report.json" || true
gzip -f "$O/soak.jsonl"
python -c "import json,sys; q=json.load(open('$O/soak.json')); print('soak', q['value'], q['attach_p99_ms'], q['attach_split_p50_ms'], q['detach_p50_ms'])"
