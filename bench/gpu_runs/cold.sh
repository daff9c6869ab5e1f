# Round 5 (profiles/r5_cold/): the cold/first-attach table on one lease, interleaved:
# --deploy processes | inprocess  x  daemons pinned | unpinned  (authz cached vs expired is the
# cold phase's two halves), then the driver's command three times.
#   gpurun --timeout 1100 -- bash bench/gpu_runs/cold.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-cold}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
run() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 300 python bench.py --gpus 1 "$@" > "$O/$name.json" 2>> "$O/bench.err" \
        || fail "$O/bench.err"
    python - "$O/$name.json" "$name" <<'PY'
import json, sys
q = json.load(open(sys.argv[1])); c = q.get("cold_attach") or {}
f = q.get("first_attach_stages_ms") or {}
print(sys.argv[2], "value", q["value"], "cold", q.get("cold_attach_p50_ms"),
      "idle", (c.get("idle_only") or {}).get("attach_p50_ms"), "first", q.get("first_attach_ms"),
      {k: f.get(k) for k in ("http.request_leg", "http.response_leg", "master.master_authz",
                             "worker")})
PY
}
PIN=$(python -c "import os; c=sorted(os.sched_getaffinity(0)); print(f'{c[len(c)//2]}:{c[len(c)//2+1]}')")
echo "pinned daemons to $PIN"
for rep in 1 2; do
    run proc_unpinned_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0
    run proc_pinned_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0 --pin "$PIN"
    run inproc_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0 --deploy inprocess
done
for i in 1 2 3; do
    run driver_$i --steps 20 --warmup 5
done
