#!/bin/bash
# Bench lines for the headline (cfg2 fp32) and the bf16 configs, a rocprofv3 kernel summary of cfg5, and the
# PMC traffic passes for the cfg5 aggregate.  Each GPU step has its own limit; any failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-round}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -5 "$OUT/$name.err"; exit $rc; }
}
run bench_cfg2 300 python bench.py
run bench_cfg2bf 300 python bench.py --config cfg2bf
run bench_cfg5 500 python bench.py --config cfg5
run prof_cfg5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --steps 5 --warmup 2
for C in FETCH_SIZE WRITE_SIZE; do
  run pmc_cfg5_$C 400 rocprofv3 --pmc $C --kernel-include-regex k_aggregate --output-format csv \
      -d "$OUT/pmc_cfg5_$C" -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 2 --warmup 1 --config cfg5
done
echo done >> "$OUT/status.txt"
