set -u
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
OUT=gpurun_out/r05b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_gat -o run -- python3 tools/extras_probe.py --only gat > $OUT/prof_gat.log 2>&1 || { echo FAIL prof_gat; tail -20 $OUT/prof_gat.log; exit 1; }
f=$(find $OUT/prof_gat -name '*kernel_stats.csv' | head -1); head -20 "$f" | cut -c1-200
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg3 -o run -- python3 bench.py --no-cpu-baseline --no-probe --no-extras > $OUT/prof_cfg3.log 2>&1 || { echo FAIL prof_cfg3; tail -20 $OUT/prof_cfg3.log; exit 1; }
f=$(find $OUT/prof_cfg3 -name '*kernel_stats.csv' | head -1); python3 tools/prof_summary.py "$f" 23 > $OUT/summary_cfg3.txt; head -20 $OUT/summary_cfg3.txt
OUT=$OUT/pmc VARIANTS="dw256pro:1 dx256:1 dx256:0" bash tools/gpu_r05_pmc.sh && python3 tools/sq_summary.py $OUT/pmc > $OUT/pmc_summary.txt; cat $OUT/pmc_summary.txt | head -60
