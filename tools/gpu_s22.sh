#!/bin/bash
# s22: bf16 rounding on v_cvt_pk_bf16_f32 (+ NaN canonicalisation): every bf16 test (bitwise vs torch rounding), the
# kernel / gemm-switch / model tests, cfg5 bench + kernel summary.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s22}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -3 "$OUT/$name.out" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step suite 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_cfg5 400 python bench.py --config cfg5 --no-cpu-baseline --no-extras
step prof_cfg5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg5" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg5.txt"; head -8 "$OUT/summary_cfg5.txt"
echo done >> "$OUT/status.txt"
