# A/B of loop_spin_us (gpumounter_amd/utils/spin.py) on one MI355X box, interleaved:
#   gpurun --timeout 900 -- bash bench/gpu_runs/spin.sh <tag>
# 1. the gRPC hop in isolation, with and without both loops polling (hop_floor.py --spin)
# 2. the driver's bench command, GM_LOOP_SPIN_US=0 vs 300, four pairs
# 3. 200 timed cycles each way, two pairs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-spin}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
for i in 1 2 3; do
    for o in "--http --tls --retry --big --shield" "--http --tls --retry --big --shield --spin"; do
        timeout -k 10 120 python bench/gpu_runs/hop_floor.py $o | tee -a "$O/hop_floor.jsonl" || exit 1
    done
done
summary() {
    python - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["value"], d["attach_p99_ms"], d["attach_split_p50_ms"],
      "detach", d["detach_p50_ms"], "probe", d["probe_quick_p50_us"])
PY
}
for i in 1 2 3 4; do
    for sp in 0 300; do
        GM_LOOP_SPIN_US=$sp timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
            > "$O/drv_${sp}_$i.json" 2> "$O/drv_${sp}_$i.err" || { tail -20 "$O/drv_${sp}_$i.err"; exit 1; }
        summary "$O/drv_${sp}_$i.json" "drv spin=$sp"
    done
done
for i in 1 2; do
    for sp in 0 300; do
        GM_LOOP_SPIN_US=$sp timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 \
            --cold-steps 0 --dump-samples "$O/long_${sp}_$i.jsonl" \
            > "$O/long_${sp}_$i.json" 2> "$O/long_${sp}_$i.err" || { tail -20 "$O/long_${sp}_$i.err"; exit 1; }
        summary "$O/long_${sp}_$i.json" "long spin=$sp"
    done
done
