# Where the emulated node keeps its kernel-backed trees (cgroupfs, container /dev): tmpfs
# (bench.py's default, as on a real node) against the working directory's disk, interleaved.
#   gpurun --timeout 900 -- bash bench/gpu_runs/node_fs.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-node_fs}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
df -T /tmp /dev/shm "$GRAFT_REPO_ROOT" > "$O/df.txt" 2>&1 || true
for i in 1 2; do
  for fs in disk tmpfs; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 20 --kernel-fs $fs \
        > "$O/${fs}_$i.json" 2> "$O/${fs}_$i.err" || fail "$O/${fs}_$i.err"
  done
done
python - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/*_?.json")):
    d = json.load(open(f))
    s = d["stage_p50_ms"]
    r = d.get("reference_emulated_same_run") or {}
    print(os.path.basename(f), d["node_fs"], "attach", d["value"], "p99", d["attach_p99_ms"],
          "detach", d["detach_p50_ms"], "mount", s["mount"], "devnodes", s["mount.devnodes"],
          "cgroup", s["mount.cgroup_rule"], "ref", r.get("attach_p50_ms"))
PY
