#!/bin/bash
# hipGraph-replay bench mode: parity test, then graph vs eager bench lines (cfg2, cfg5).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-graph}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -20 "$OUT/$name.err"; exit $rc; }
}
run test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_model.py -k captured
run bench_graph 300 python bench.py --no-cpu-baseline
run bench_eager 300 python bench.py --no-cpu-baseline --eager
run bench_graph_noprobe 300 python bench.py --no-cpu-baseline --no-probe
if [ "${CFG5:-0}" = "1" ]; then
  run bench5_graph 600 python bench.py --no-cpu-baseline --config cfg5 --steps 10
fi
echo done >> "$OUT/status.txt"
