#!/bin/bash
# rocprofv3 kernel-trace summaries of the bench command (no probe, no extras, no CPU baseline) for CONFIGS,
# optionally preceded by full bench lines (BENCH=1).  Each GPU step has its own limit; any failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -20 "$OUT/$name.err"; exit $rc; }
}
for C in ${CONFIGS:-cfg3}; do
  if [ "${BENCH:-0}" = "1" ]; then run bench_$C 600 python bench.py --config $C ${BENCH_ARGS:-}; fi
  run prof_$C 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
      python3 bench.py --config $C --no-cpu-baseline --no-probe --no-extras ${BENCH_ARGS:-}
  f=$(ls "$OUT"/prof_$C/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find "$OUT/prof_$C" -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_$C.txt"
  head -25 "$OUT/summary_$C.txt"
done
echo done >> "$OUT/status.txt"
