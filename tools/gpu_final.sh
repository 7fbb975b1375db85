#!/bin/bash
# Final-tree evidence: full GPU suite + smoke, the driver's bench command (cfg3 headline with extras.cfg5 / batches and
# the CPU baseline), then per config (cfg3, cfg5 bf16): the rocprofv3 kernel-trace summary of the bench command (no
# probe / extras / CPU baseline) and the aggregate family's PMC FETCH_SIZE / WRITE_SIZE in separate passes.  Every step
# time-limited; stop at the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.out" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
# SUITE=0 / EVID=0 skip a half (one gpurun call is at most 20 minutes: the suite and the evidence go in separate calls)
if [ "${SUITE:-1}" = "1" ]; then
  step suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
fi
[ "${EVID:-1}" = "1" ] || { echo done >> "$OUT/status.txt"; exit 0; }
step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
step prof_batches 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_batches" -o run -- \
    python3 tools/batches_prof.py --steps 200
for C in cfg3 cfg5; do
  step prof_$C 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
      python3 bench.py --config $C --no-cpu-baseline --no-probe --no-extras
  f=$(find "$OUT/prof_$C" -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_$C.txt"; head -6 "$OUT/summary_$C.txt"
  for K in FETCH_SIZE WRITE_SIZE; do
    step pmc_${K}_$C 300 rocprofv3 --pmc $K --kernel-include-regex "k_agg" --output-format csv -d "$OUT/pmc_${K}_$C" \
        -o run -- python3 bench.py --config $C --no-cpu-baseline --no-probe --no-extras --steps 2 --warmup 1
  done
done
echo done >> "$OUT/status.txt"
