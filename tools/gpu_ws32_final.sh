#!/bin/bash
# HEAD with k_ws_f32: the GPU parity suite, smoke(), the default bench line, and the rocprofv3 kernel-trace summary
# of the same cfg3 command (no probe) for profiles/r02.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ws32_final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -30 "$OUT/$name.log"; exit $rc ;; esac
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --no-probe
echo done >> "$OUT/status.txt"
tail -2 "$OUT/pytest_gpu.log"; tail -1 "$OUT/smoke.log"; tail -1 "$OUT/bench.log" | cut -c1-300
