set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r12
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for n in default zero pool; do
  case $n in default) a="";; zero) a="--steps 300 --warmup 30";; pool) a="--steps 300 --warmup 30 --warm-pool 1";; esac
  timeout -k 10 300 python bench.py $a > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['attach_p99_ms'], d['detach_p50_ms'], d['detach_p99_ms'], d['stage_p50_ms'], d.get('reference_emulated_same_run'))"
done
