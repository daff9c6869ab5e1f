# First-request authz A/B on one lease (profiles/r5_cold/): the self-review on and off,
# interleaved, daemons pinned; first attach and cold attach split.
#   gpurun --timeout 1100 -- bash bench/gpu_runs/authz_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-authz_ab}
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
      "cold authz", (c.get("stage_p50_ms") or {}).get("master_authz"),
      "idle", (c.get("idle_only") or {}).get("attach_p50_ms"), "first", q.get("first_attach_ms"),
      {k: f.get(k) for k in ("http.request_leg", "http.response_leg", "master.master_authz",
                             "worker")})
PY
}
PIN=$(python -c "import os; c=sorted(os.sched_getaffinity(0)); print(f'{c[len(c)//2]}:{c[len(c)//2+1]}')")
echo "pinned daemons to $PIN"
for rep in 1 2 3 4; do
    run self_on_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0 --pin "$PIN"
    run self_off_$rep --steps 20 --warmup 5 --cold-steps 10 --call-cycles 0 --pin "$PIN" \
        --daemon-env GM_AUTHZ_SELF_REVIEW=false
done
