#!/bin/bash
# A/B of the fp32 NT GEMM modes on the cfg3 shapes (tools/h2_bench.py), each setting in its own process.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-h2ab}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python tools/h2_bench.py > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; cat "$OUT/$name.out"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -20 "$OUT/$name.err"; exit $rc; }
}
run split HGIN_F32_GEMM=split
run split_tiled HGIN_NT_WS32=0
run h2_occ2 HGIN_F32_GEMM=h2 HGIN_H2_OCC=2
run h2_occ3 HGIN_F32_GEMM=h2 HGIN_H2_OCC=3
