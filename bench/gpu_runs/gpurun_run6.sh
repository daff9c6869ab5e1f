set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -k "hbm" -v -s --timeout 120 --timeout-method thread > $O/pytest_hbm.log 2>&1 || { tail -30 $O/pytest_hbm.log; exit 1; }
grep -E "HBM|passed|failed" $O/pytest_hbm.log
timeout -k 10 400 python -u bench/probe_sweep.py > $O/probe_sweep.json 2> $O/probe_sweep.err || { tail -30 $O/probe_sweep.err; exit 1; }
cat $O/probe_sweep.json
