set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r14
mkdir -p $O
timeout -k 10 400 python -u bench/probe_sweep.py --quick > $O/probe_sweep_quick.json 2> $O/probe_sweep_quick.err || { tail -20 $O/probe_sweep_quick.err; exit 1; }
python -c "
import json; d=json.load(open('$O/probe_sweep_quick.json')); print(json.dumps(d['hbm_copy_GBps'], indent=0)); print(d['hbm_read_GBps']); print(d['torch'])"
