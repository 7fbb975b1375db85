#!/bin/bash
# s23: single-pass PReLU-fused dW at N = 128, K = 512 (the readout's first Linear): kernel / model / bf16 tests, cfg3 and
# cfg5 kernel summaries.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s23}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.out" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bf16.py tests/test_gpu_readout_loss.py tests/test_gpu_variants.py -x -q --timeout 300 --timeout-method thread
for C in cfg3 cfg5; do
  step prof_$C 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
      python3 bench.py --config $C --no-cpu-baseline --no-probe --no-extras
  f=$(find "$OUT/prof_$C" -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_$C.txt"; grep -E "k_wsd|total" "$OUT/summary_$C.txt"
done
echo done >> "$OUT/status.txt"
