set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r11
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "validate_tool" -v -s --timeout 240 --timeout-method thread > $O/pytest_validate.log 2>&1 || { tail -40 $O/pytest_validate.log; exit 1; }
grep -E "allreduce|passed|failed|busbw" $O/pytest_validate.log | tail -5
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --latency realistic --warm-pool 1 > $O/realistic_pool.json 2> $O/realistic_pool.err || { tail -20 $O/realistic_pool.err; exit 1; }
python -c "
import json; d=json.load(open('$O/realistic_pool.json')); print('realistic+pool', d['value'], d['attach_p99_ms'], d['detach_p50_ms'], d['config']['deploy'])"
