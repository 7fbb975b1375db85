#!/bin/bash
# round 6: the plain fp32 dX GEMM at N = 256 (the readout's K = 128) as k_wss_f32 EPI 5 — switch / model suites, the
# A/B against tools/ab/libhgin_base.so (the tiled kernel for these shapes), then cfg3 with a kernel summary
set -u
OUT=gpurun_out/${TAG:-r06w}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -2 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; grep -E "^E |FAILED|Error" "$OUT/$name.log" | head -30; exit $rc; }
}
step tests 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gemm_switch.py tests/test_gpu_model.py
for rep in 1 2; do
  for L in new base; do
    A=""; [ $L = base ] && A="--lib tools/ab/libhgin_base.so"
    step ab_${rep}_$L 120 python -u tools/gemm_ab.py --M 6000000 --reps 10 --only dxro,dx256p $A
    grep '^{' "$OUT/ab_${rep}_$L.log" >> "$OUT/ab_plain.txt"
  done
done
step prof_cfg3 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
    python3 bench.py --config cfg3 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg3" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg3.txt"; head -24 "$OUT/summary_cfg3.txt"
