#!/bin/bash
# Round-3 s14: cfg3 with the tiled PReLU-fused dW (g_z stored by the first K tile) in place of k_wsd_f32<..., PRO>
# (HGIN_TN_WS=0): bench line + kernel summary of the same command.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s14}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -c 600 "$OUT/$name.out"; echo
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
export HGIN_TN_WS=0
step prof_cfg3 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
    python3 bench.py --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg3" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg3.txt"; head -16 "$OUT/summary_cfg3.txt"
echo done >> "$OUT/status.txt"
