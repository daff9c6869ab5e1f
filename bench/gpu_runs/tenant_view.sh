# Tenant-side view on the GPU box: the GPU tests that exercise it, then a short default bench
# whose JSON carries "tenant_view".   gpurun --timeout 700 -- bash bench/gpu_runs/tenant_view.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "tenant_side or busy_detection or e2e_attach" > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -5 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/default.json 2> $O/default.err || { tail -30 $O/default.err; exit 1; }
python -c "import json; d=json.load(open('$O/default.json')); print(d['value'], d['tenant_view'])"
