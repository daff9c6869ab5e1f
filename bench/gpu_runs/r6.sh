# Round-6 re-measurement on one MI355X box, from the repository root:
#   gpurun --timeout 1150 -- bash bench/gpu_runs/r6.sh <tag>
# 1. the driver's command twice (default bench.py: attach p50, cold phase interleaved A/B on one
#    master process, first attach);
# 2. the warm pool with standbys at the floor class (default) and with the low pool class
#    (GM_POOL_PRIORITY_CLASS=gpumounter-standby: each attach yields the only standby GPU);
# 3. attach latency at 1/2/4/8 GPUs per Pod (mock 8-GPU inventory) and at 1 on the real GPU.
# Every GPU step has its own time limit; the first failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for i in 1 2; do
    timeout -k 10 300 python bench.py > "$O/default_$i.json" 2> "$O/default_$i.err" \
        || fail "$O/default_$i.err"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --warm-pool 1 \
    > "$O/pool_floor.json" 2> "$O/pool_floor.err" || fail "$O/pool_floor.err"
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 --warm-pool 1 \
    --daemon-env GM_POOL_PRIORITY_CLASS=gpumounter-standby \
    > "$O/pool_low.json" 2> "$O/pool_low.err" || fail "$O/pool_low.err"
for n in 1 2 4 8; do
    timeout -k 10 240 python bench.py --amdsmi mock --gpus $n --steps 100 --warmup 20 \
        --cold-steps 0 > "$O/mock_n$n.json" 2> "$O/mock_n$n.err" || fail "$O/mock_n$n.err"
done
python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("default_1", "default_2", "pool_floor", "pool_low", "mock_n1", "mock_n2", "mock_n4",
          "mock_n8"):
    d = json.load(open(f"{o}/{f}.json"))
    c = d.get("cold_attach") or {}
    print(f, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], "cold", c.get("attach_p50_ms"),
          "idle", (c.get("idle_only") or {}).get("attach_p50_ms"), "first",
          d.get("first_attach_ms"), "split", d.get("attach_split_p50_ms"))
PY
