#!/bin/bash
# round 6: bf16 z-from-y (hgin_gin_mlp_fwd_zy_bf16 / hgin_gin_mlp_bwd_w_zy_bf16): the bf16 suite, the model suites, the
# cfg5 step time and kernel summary
set -u
OUT=gpurun_out/${TAG:-r06k}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; grep -E "^E |FAILED|Error" "$OUT/$name.log" | head -30; exit $rc; }
}
step bf16 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py
step model 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_readout_loss.py tests/test_gpu_store.py
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg5" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg5.txt"; head -16 "$OUT/summary_cfg5.txt"; tail -2 "$OUT/summary_cfg5.txt"
step full5 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py -k cfg5
step bench5 300 python bench.py --config cfg5 --no-cpu-baseline --no-extras --steps 20 --warmup 3
# the fused HetroGAT step with its folds / W_s staged in LDS
step gat 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smallbatch_gat.py
step sbgat 120 python -u tools/sb_prof.py --steps 200 --gat
cat "$OUT/sbgat.log" | grep ms_per_batch
step trgat 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_gat" -o run -- python3 tools/sb_prof.py --steps 200 --gat
python3 tools/sb_busy.py "$OUT/trace_gat" --steps 200 --label gat > "$OUT/sb_busy_gat.json" && head -20 "$OUT/sb_busy_gat.json"
