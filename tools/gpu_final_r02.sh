#!/bin/bash
# Round-2 HEAD evidence: the GPU parity suite, smoke(), the default bench line (cfg3), cfg5, and cfg3 with the
# dead relations pruned (reported separately).  Each GPU step has its own limit; anything but
# pass / ordinary test failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-final_r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0|1) ;; *) echo "FATAL $name $rc"; tail -20 "$OUT/$name.log"; exit $rc ;; esac
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py
step bench_cfg5 400 python bench.py --config cfg5 --no-cpu-baseline
step bench_cfg3_pruned 400 python bench.py --prune-dead --no-cpu-baseline --no-extras
echo done >> "$OUT/status.txt"
tail -3 "$OUT/pytest_gpu.log"; tail -1 "$OUT/smoke.log"
