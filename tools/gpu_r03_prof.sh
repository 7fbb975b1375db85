#!/bin/bash
# Round-3 evidence: bench lines (CONFIGS), rocprofv3 kernel summaries of the same bench commands (no probe / extras /
# CPU baseline), PMC FETCH_SIZE / WRITE_SIZE passes for the cfg3 aggregate family.  Each step time-limited.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -20 "$OUT/$name.err"; exit $rc; }
}
for C in ${BENCH_CONFIGS:-cfg5}; do run bench_$C 600 python bench.py --config $C; done
for C in ${PROF_CONFIGS:-cfg3 cfg5}; do
  run prof_$C 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
      python3 bench.py --config $C --no-cpu-baseline --no-probe --no-extras
  f=$(find "$OUT/prof_$C" -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_$C.txt"
  head -30 "$OUT/summary_$C.txt"
done
if [ "${PMC:-1}" = "1" ]; then
  for K in FETCH_SIZE WRITE_SIZE; do
    run pmc_$K 300 rocprofv3 --pmc $K --kernel-include-regex "k_agg" --output-format csv -d "$OUT/pmc_$K" -o run -- \
        python3 bench.py --no-cpu-baseline --no-probe --no-extras --steps 2 --warmup 1
  done
fi
echo done >> "$OUT/status.txt"
