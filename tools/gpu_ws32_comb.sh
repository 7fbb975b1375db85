#!/bin/bash
# k_ws_f32 with the dX combine epilogue: GEMM switch tests, the micro-benchmark with / without, the full GPU suite,
# smoke() and the cfg3 bench line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ws32_comb}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -30 "$OUT/$name.log"; exit $rc ;; esac
}
step switch 500 python -u -m pytest tests/test_gpu_gemm_switch.py -x -v --timeout 400 --timeout-method thread
step bench_ws 300 python tools/ws32_bench.py
HGIN_NT_WS32=0 step bench_tiled 300 python tools/ws32_bench.py
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python bench.py
echo done >> "$OUT/status.txt"
cat "$OUT/bench_ws.log" "$OUT/bench_tiled.log" | grep HGIN; tail -1 "$OUT/pytest_gpu.log"; tail -1 "$OUT/bench.log" | cut -c1-300
