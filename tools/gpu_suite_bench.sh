#!/bin/bash
# Full GPU suite, then bench lines (cfg3 headline + optional others).  Each GPU step under its own limit; a
# failure, abort or timeout ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-suite}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -30 "$OUT/$name.err"; exit $rc; }
}
echo "start $(date)" > "$OUT/status.txt"
if [ "${SUITE:-1}" = "1" ]; then
  run pytest_gpu ${PYTEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rP
fi
for C in ${CONFIGS:-cfg3}; do
  run bench_$C 600 python bench.py --config $C ${BENCH_ARGS:-}
done
echo "done $(date)" >> "$OUT/status.txt"
tail -3 "$OUT/pytest_gpu.out" 2>/dev/null
for C in ${CONFIGS:-cfg3}; do cat "$OUT/bench_$C.out"; done
