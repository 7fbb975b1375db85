#!/bin/bash
# Round-end evidence for one config: the bench line, the rocprofv3 kernel-trace summary of the SAME bench
# command (no probe), and the PMC traffic of the aggregate family in separate FETCH_SIZE / WRITE_SIZE passes.
set -u
cd "$(dirname "$0")/.."
CFG=${CFG:-cfg2}
OUT=gpurun_out/final_$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -5 "$OUT/$name.err"; exit $rc; }
}
run bench 600 python bench.py --config $CFG ${BENCH_ARGS:-}
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --config $CFG --no-cpu-baseline --no-probe
for C in FETCH_SIZE WRITE_SIZE; do
  run pmc_$C 600 rocprofv3 --pmc $C --kernel-include-regex k_agg --output-format csv -d "$OUT/pmc_$C" -o run -- \
      python3 bench.py --no-cpu-baseline --no-probe --steps 2 --warmup 1 --config $CFG
done
echo done >> "$OUT/status.txt"
