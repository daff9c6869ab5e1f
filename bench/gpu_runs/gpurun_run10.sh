set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r10
mkdir -p $O
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --latency realistic --protocol reference > $O/ref_realistic.json 2> $O/ref_realistic.err || { tail -20 $O/ref_realistic.err; exit 1; }
cut -c1-300 $O/ref_realistic.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d "$R/$O/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 10 --ref-steps 0 > "$R/$O/prof.log" 2>&1; echo "rocprof rc=$?"
find "$R/$O/prof" -name "*stats.csv"
