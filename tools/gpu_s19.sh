#!/bin/bash
# s19: bf16 first layer with (1 + eps) folded into the weight operand: bf16 / model / dist / fullsize-bf16 tests,
# cfg5 bench line + kernel summary.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s19}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -3 "$OUT/$name.out" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step tests 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_model.py tests/test_gpu_dist.py tests/test_gpu_store.py "tests/test_gpu_fullsize.py::test_cfg5_bf16_vs_cfg3_fp32_full_size" -x -q -s --timeout 300 --timeout-method thread
step bench_cfg5 400 python bench.py --config cfg5 --no-cpu-baseline --no-extras
step prof_cfg5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg5" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg5.txt"; head -12 "$OUT/summary_cfg5.txt"
echo done >> "$OUT/status.txt"
