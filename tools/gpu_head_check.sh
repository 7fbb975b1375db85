#!/bin/bash
# HEAD verification on a fresh box: the GPU parity suite, smoke(), and the default bench line.
# Every GPU step has its own limit; anything but pass / ordinary test failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-head}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0|1) ;; *) echo "FATAL $name $rc"; tail -20 "$OUT/$name.log"; exit $rc ;; esac
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py
echo done >> "$OUT/status.txt"
tail -3 "$OUT/pytest_gpu.log"; tail -1 "$OUT/smoke.log"; cat "$OUT/bench.log" | tail -1
