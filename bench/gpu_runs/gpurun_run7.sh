set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r7
mkdir -p $O
for sc in scale contention soak; do
  timeout -k 10 300 python bench/configs.py $sc > $O/${sc}_mock.json 2> $O/${sc}_mock.err || { tail -20 $O/${sc}_mock.err; exit 1; }
  echo "$sc mock: $(cut -c1-300 $O/${sc}_mock.json)"
done
timeout -k 10 400 python bench/configs.py soak --amdsmi "" > $O/soak_real.json 2> $O/soak_real.err || { tail -20 $O/soak_real.err; exit 1; }
echo "soak real: $(cut -c1-400 $O/soak_real.json)"
