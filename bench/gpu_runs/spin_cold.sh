# Cold attaches with and without loop polling (loop_spin_us), interleaved, on one MI355X box:
#   gpurun --timeout 900 -- bash bench/gpu_runs/spin_cold.sh <tag>
# Each run: the driver's timed loop, then 30 attaches after 0.3 s of idleness each (authz answers
# expired), so the cold median rests on 30 samples per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-spin_cold}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
for i in 1 2 3; do
    for sp in 0 300; do
        GM_LOOP_SPIN_US=$sp timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
            --cold-steps 30 > "$O/cold_${sp}_$i.json" 2> "$O/cold_${sp}_$i.err" \
            || { tail -20 "$O/cold_${sp}_$i.err"; exit 1; }
        python - "$O/cold_${sp}_$i.json" "$sp" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["cold_attach"] or {}
print("spin", sys.argv[2], "warm", d["value"], "p99", d["attach_p99_ms"], "cold", d["cold_attach_p50_ms"],
      "idle_only", c.get("idle_only", {}).get("attach_p50_ms"), "load", d["box"]["loadavg_1m"])
PY
    done
done
