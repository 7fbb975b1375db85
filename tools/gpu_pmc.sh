#!/bin/bash
# Hardware-counter passes for the aggregate kernel: FETCH_SIZE and WRITE_SIZE in SEPARATE rocprofv3 runs
# (kernel-trace only alongside; never with sys/runtime trace), then the per-launch traffic summary.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc}
CFG=${CFG:-cfg2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $C --kernel-include-regex k_aggregate --output-format csv \
    -d "$OUT/$C" -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 3 --warmup 1 --config $CFG \
    > "$OUT/$C.log" 2>&1
  rc=$?; echo "$C $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || exit $rc
done
