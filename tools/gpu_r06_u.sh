#!/bin/bash
# round 6: the bf16 readout tail (zy only for the weight-stationary shapes, 32-wide K tiles for the K = 32 dX) —
# the model / bf16 / full-size suites, then cfg5 with a kernel summary
set -u
OUT=gpurun_out/${TAG:-r06u}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; grep -E "^E |FAILED|Error" "$OUT/$name.log" | head -30; exit $rc; }
}
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_bf16.py \
  tests/test_gpu_fullsize.py tests/test_gpu_store.py tests/test_gpu_dist.py tests/test_gpu_variants.py tests/test_gpu_readout_loss.py
for C in cfg5; do
  step prof_$C 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
      python3 bench.py --config $C --no-cpu-baseline --no-probe --no-extras
  f=$(find "$OUT/prof_$C" -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_$C.txt"; head -8 "$OUT/summary_$C.txt"; tail -2 "$OUT/summary_$C.txt"
done
