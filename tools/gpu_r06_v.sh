#!/bin/bash
# round 6: the readout's K = 512, N = 128 bf16 forward with two workgroups per CU (k_ws_bf16 ",wpc2") — bf16 / switch
# suites, the forward A/B against tools/ab/libhgin_base.so (one workgroup per CU), then cfg5 with a kernel summary
set -u
OUT=gpurun_out/${TAG:-r06v}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; grep -E "^E |FAILED|Error" "$OUT/$name.log" | head -30; exit $rc; }
}
step tests 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_gemm_switch.py
for rep in 1 2; do
  for L in new base; do
    A=""; [ $L = base ] && A="--lib tools/ab/libhgin_base.so"
    step ab_${rep}_$L 120 python -u tools/gemm_ab.py --dtype bf16 --M 6000000 --reps 10 --only fwdro,fwd512 $A
    grep '^{' "$OUT/ab_${rep}_$L.log" >> "$OUT/ab_wpc2.txt"
  done
done
step prof_cfg5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg5" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg5.txt"; head -12 "$OUT/summary_cfg5.txt"; tail -2 "$OUT/summary_cfg5.txt"
