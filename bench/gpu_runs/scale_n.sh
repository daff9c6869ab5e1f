# Attach latency at 1/2/4/8 GPUs per Pod on one box (BASELINE: "scale one Pod 1→8"). The box has
# one GPU, so N>1 runs on the bundled 8×MI355X mock inventory (control plane + emulated node ops,
# no tenant-side GPU check); N=1 also runs on the real libamd_smi inventory for comparison.
#   gpurun --timeout 900 -- bash bench/gpu_runs/scale_n.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-scale_n}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
for n in 1 2 4 8; do
    timeout -k 10 240 python bench.py --amdsmi mock --gpus $n --steps 100 --warmup 20 \
        > "$O/mock_n$n.json" 2> "$O/mock_n$n.err" || fail "$O/mock_n$n.err"
done
timeout -k 10 240 python bench.py --gpus 1 --steps 100 --warmup 20 > "$O/real_n1.json" \
    2> "$O/real_n1.err" || fail "$O/real_n1.err"
python - "$O" <<'PY'
import json, sys
for f in ("mock_n1", "mock_n2", "mock_n4", "mock_n8", "real_n1"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    ref = d.get("reference_emulated_same_run") or {}
    print(f, d["value"], d["attach_p99_ms"], d["detach_p50_ms"], ref.get("attach_p50_ms"),
          {k: v for k, v in d["stage_p50_ms"].items() if v >= 0.05})
PY
