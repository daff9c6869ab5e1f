set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/$O/counters_list.txt" 2>&1; echo "list rc=$?"
grep -o -E "(FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE|SQ_VALU_MFMA_BUSY_CYCLES|SQ_BUSY_CYCLES|SQ_WAVE_CYCLES|SQ_INSTS_VALU_MFMA_MOPS_BF16)" "$R/$O/counters_list.txt" | sort | uniq -c
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/$O/p1" -o p1 -- python3 "$R/bench/pmc_probe.py" > "$R/$O/p1.log" 2>&1; echo "p1 rc=$?"; tail -2 "$R/$O/p1.log"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/$O/p2" -o p2 -- python3 "$R/bench/pmc_probe.py" > "$R/$O/p2.log" 2>&1; echo "p2 rc=$?"; tail -2 "$R/$O/p2.log"
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/$O/p3" -o p3 -- python3 "$R/bench/pmc_probe.py" > "$R/$O/p3.log" 2>&1; echo "p3 rc=$?"; tail -2 "$R/$O/p3.log"
find "$R/$O" -name "*.csv" | head -20
