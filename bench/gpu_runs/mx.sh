# Block-scaled (MX) MFMA probe on one MI355X: lane-map discovery with one-hot data, the fp8
# tile numerics check, and the fp8/fp4 register-resident peaks (bf16 peak alongside).
#   gpurun --timeout 600 -- bash bench/gpu_runs/mx.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-mx}
mkdir -p "$O"
fail() { tail -40 "$1"; exit 1; }
timeout -k 10 120 python bench/mx_layout.py > "$O/layout.json" 2> "$O/layout.err" || fail "$O/layout.err"
cat "$O/layout.json"
timeout -k 10 180 python - > "$O/mx.json" 2> "$O/mx.err" <<'PY' || fail "$O/mx.err"
import json
import numpy as np
from gpumounter_amd.ops import mx, probe
out = {"check_fp8": [mx.check_fp8(0, s) for s in range(3)]}
for fmt in ("fp8", "fp4"):
    runs = [mx.peak(0, fmt, 20000) for _ in range(3)]
    out[fmt] = {"tflops": [round(t, 1) for t, _ in runs],
                "bitwise_equal_runs": all(np.array_equal(runs[0][1].view(np.uint32),
                                                         r[1].view(np.uint32)) for _, r in runs),
                "finite": bool(np.all(np.isfinite(runs[0][1])))}
out["bf16_tflops"] = round(probe.mfma_tflops(0), 1)
print(json.dumps(out))
PY
cat "$O/mx.json"
