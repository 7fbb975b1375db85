#!/bin/bash
# s24: k_wsd_bf16 with hoistable per-lane DMA offsets: dW tests (bitwise), timing of the PRO / plain dW at M = 6M, cfg5 bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s24}
mkdir -p "$OUT"
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.out" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py tests/test_gpu_gemm_switch.py -x -q --timeout 300 --timeout-method thread
step t_pro 120 python tools/wsd_one.py bf16 pro 6000000
step t_plain 120 python tools/wsd_one.py bf16 plain 6000000
step bench_cfg5 400 python bench.py --config cfg5 --no-cpu-baseline --no-extras
echo done >> "$OUT/status.txt"
