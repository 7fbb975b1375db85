#!/bin/bash
# fp32 weight-stationary forward GEMM (k_ws_f32): the GEMM switch tests (bit-identical to the tiled kernel), the
# kernel micro-benchmark with and without it, then the cfg3 bench line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ws32}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -30 "$OUT/$name.log"; exit $rc ;; esac
}
step switch 500 python -u -m pytest tests/test_gpu_gemm_switch.py -x -v --timeout 400 --timeout-method thread
step bench_ws 200 python tools/ws32_bench.py
HGIN_NT_WS32=0 step bench_tiled 200 python tools/ws32_bench.py
step bench_cfg3 400 python bench.py --no-cpu-baseline --no-extras
echo done >> "$OUT/status.txt"
cat "$OUT/bench_ws.log" "$OUT/bench_tiled.log"; tail -1 "$OUT/bench_cfg3.log" | cut -c1-400
