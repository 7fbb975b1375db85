#!/bin/bash
# s18: k_wsd_f32 refills a block's slot right after its split pass: dW tests, model tests, cfg3 bench + kernel summary.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s18}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -3 "$OUT/$name.out" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_variants.py -x -q --timeout 300 --timeout-method thread
step prof_cfg3 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
    python3 bench.py --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg3" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg3.txt"; head -12 "$OUT/summary_cfg3.txt"
echo done >> "$OUT/status.txt"
