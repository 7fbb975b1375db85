#!/bin/bash
# round 6: the fp32 K = 512 first-layer forward as two k_wss_f32 passes — bitwise against the tiled kernel
# (test_gpu_gemm_switch), the model / variant suites, per-launch A/B at M = 3M, and the cfg3 step with its kernel summary
set -u
OUT=gpurun_out/${TAG:-r06i}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; grep -E "^E |FAILED|Error" "$OUT/$name.log" | head -20; exit $rc; }
}
step switch 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_gemm_switch.py
step model 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_variants.py tests/test_gpu_readout_loss.py
step ab 300 bash -c 'for r in 1 2; do python -u tools/gemm_ab.py --M 3000000 --reps 10 --only fwd512,fwd512acc,fwd256; done'
grep '^{' "$OUT/ab.log"
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
    python3 bench.py --config cfg3 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg3" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg3.txt"; head -12 "$OUT/summary_cfg3.txt"
