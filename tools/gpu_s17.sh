#!/bin/bash
# s17: bf16 K = 512 forward with the eps-scaling pass over the self half only: GEMM switch tests (bitwise across kernels),
# bf16 model tests, timing A/B, cfg5 bench line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s17}
mkdir -p "$OUT"
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -4 "$OUT/$name.out" | cut -c1-400
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step sw 600 python -u -m pytest tests/test_gpu_gemm_switch.py tests/test_gpu_bf16.py -x -q --timeout 400 --timeout-method thread
step eps_ab 200 python tools/ws_bf16_eps_ab.py
step bench_cfg5 400 python bench.py --config cfg5 --no-cpu-baseline --no-extras
echo done >> "$OUT/status.txt"
