#!/bin/bash
# Run named GPU steps in order, each under its own time limit, stopping at the first failure.
#   OUT=gpurun_out/x tools/gpu_steps.sh 'name|seconds|command' ...
# Each step's stdout / stderr go to $OUT/<name>.out / .err; $OUT/status.txt records the exit codes.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/steps}
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; lim=${rest%%|*}; cmd=${rest#*|}
  echo "== $name (limit ${lim}s): $cmd"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?
  echo "$name $rc" >> "$OUT/status.txt"
  tail -3 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then echo "FATAL $name rc=$rc"; tail -20 "$OUT/$name.err"; exit $rc; fi
done
echo "all steps ok"
