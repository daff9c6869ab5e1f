# rocprofv3 kernel + marker trace at the round-5 tree (profiles/r5_rocprof/): the in-process
# deployment (gm:* worker and gm:master_* ranges land in one trace) and the driver's process
# deployment (the daemons inherit the profiler's preload: roctx ranges on), with --stats.
#   gpurun --timeout 900 -- bash bench/gpu_runs/rocprof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-rocprof}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -f csv -d "$O/inproc" -o bench \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --deploy inprocess --steps 50 --warmup 10 --cold-steps 0 \
    --call-cycles 0 > "$O/inproc.log" 2>&1 || fail "$O/inproc.log"
echo inproc-ok
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -f csv -d "$O/procs" -o bench \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --cold-steps 0 --call-cycles 0 \
    > "$O/procs.log" 2>&1 || fail "$O/procs.log"
echo procs-ok
find "$O" -name "*_stats.csv" | sort
