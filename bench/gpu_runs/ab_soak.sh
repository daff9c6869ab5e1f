# Same-box A/B of two trees on bench/configs.py soak (real libamd_smi inventory, in-process
# deployment), interleaved:
#   gpurun --timeout 900 -- bash bench/gpu_runs/ab_soak.sh <tag> <treeA> <treeB> [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab_soak}
A=${2:-ab/base}
B=${3:-ab/head}
ROUNDS=${4:-3}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
for i in $(seq 1 "$ROUNDS"); do
    for t in "$A" "$B"; do
        n=$(basename "$t")_$i
        timeout -k 10 60 python3 -m gpumounter_amd.utils.calib > "$O/$n.calib.json" || exit 1
        (cd "$t" && timeout -k 10 240 python3 bench/configs.py soak --amdsmi "" > "$O/$n.json" \
            2> "$O/$n.err") || { tail -30 "$O/$n.err"; exit 1; }
        echo "$n $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['attach_p50_ms'], d['attach_p99_ms'], d.get('detach_p50_ms'))" "$O/$n.json")"
    done
done
