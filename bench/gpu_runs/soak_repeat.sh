# The 1000-cycle soak on the real inventory, three times back to back (run-to-run tail spread).
#   gpurun --timeout 600 -- bash bench/gpu_runs/soak_repeat.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-soak_repeat}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for i in 1 2 3; do
  timeout -k 10 240 python bench/configs.py soak --amdsmi "" > "$O/soak_real_$i.json" \
      2> "$O/soak_real_$i.err" || fail "$O/soak_real_$i.err"
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['attach_p50_ms'], d['attach_p99_ms'], d['detach_p50_ms'], d['detach_p99_ms'], d['orphaned_cgroup_entries'], d['orphaned_device_nodes'])" "$O/soak_real_$i.json"
done
