# Same-box A/B of two source trees with the driver's exact bench command, interleaved, with the
# box calibration (gpumounter_amd/utils/calib.py) before every run:
#   gpurun --timeout 900 -- bash bench/gpu_runs/ab.sh <tag> <treeA> <treeB> [rounds]
# <treeX> are directories holding a `git archive` of the commit and its built native libraries
# (e.g. ab/r2 = 03e2ccc, ab/head = HEAD). Results: gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
A=${2:-ab/r2}
B=${3:-ab/head}
ROUNDS=${4:-3}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
for i in $(seq 1 "$ROUNDS"); do
    for t in "$A" "$B"; do
        n=$(basename "$t")_$i
        timeout -k 10 60 python3 -m gpumounter_amd.utils.calib > "$O/$n.calib.json" || exit 1
        (cd "$t" && timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
            --dump-samples "$O/$n.samples.jsonl" > "$O/$n.json" 2> "$O/$n.err") || { tail -30 "$O/$n.err"; exit 1; }
        echo "$n $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d.get('attach_split_p50_ms'), d['probe_quick_p50_us'], d.get('cold_attach_p50_ms'), (d.get('box') or {}).get('grpc_rtt_us'))" "$O/$n.json")"
    done
done
# the builder's own longer command, once per tree
for t in "$A" "$B"; do
    n=$(basename "$t")_long
    (cd "$t" && timeout -k 10 300 python3 bench.py --gpus 1 --steps 100 --warmup 20 --ref-steps 0 \
        > "$O/$n.json" 2> "$O/$n.err") || { tail -30 "$O/$n.err"; exit 1; }
    echo "$n $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d.get('attach_split_p50_ms'), d['probe_quick_p50_us'])" "$O/$n.json")"
done
