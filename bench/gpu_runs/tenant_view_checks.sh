# The tenant-side view and force-removal GPU tests, verbose (-s keeps their printed numbers).
#   gpurun --timeout 500 -- bash bench/gpu_runs/tenant_view_checks.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_tv2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -s --timeout 200 --timeout-method thread -k "tenant_view_needs or tenant_side or force_remove_waits" > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
grep -E "PASSED|FAILED|kfd only|tenant view|force removal" $O/gpu_tests.log
