#!/bin/bash
# Round-3 s10: the 128 x 256 NT tiles (HGIN_NT_TN4=1 register-staged, =2 software pipeline k_nt_pipe) — bitwise
# parity against the default through the GEMM switch child, then A/B timing on the cfg3 shapes.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s10}
mkdir -p "$OUT"
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -6 "$OUT/$name.out"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step tests 600 python -u -m pytest tests/test_gpu_gemm_switch.py -x -q --timeout 400 --timeout-method thread
step ab_default 240 python tools/h2_bench.py
step ab_tn4 240 env HGIN_NT_TN4=1 python tools/h2_bench.py
step ab_pipe 240 env HGIN_NT_TN4=2 python tools/h2_bench.py
echo done >> "$OUT/status.txt"
