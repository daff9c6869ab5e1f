# An every-mode chaos sweep (bench/chaos_sweep.py) on a GPU box's CPU share, 8 runs at a time:
#   gpurun --timeout 1150 -- bash bench/gpu_runs/chaos_box.sh <tag> <seed> [<seed> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 1080 python bench/chaos_sweep.py --seeds "$@" --jobs 8 --timeout 600 --out "$O" \
    > "$O/sweep.log" 2>&1
rc=$?
tail -3 "$O/sweep.log"
exit $rc
