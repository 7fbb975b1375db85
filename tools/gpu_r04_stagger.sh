#!/bin/bash
# Round 4: the staggered fp32 forward (k_wss_f32, HGIN_WS_STAGGER = 1) — bitwise switch tests, then per-launch time at
# the cfg3 shape against k_ws_f32 (tools/gemm_ab.py), then a cfg3 bench line with it on.  Each GPU step time-limited.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04s}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc $(date +%T)" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -30 "$OUT/$name.err"; exit $rc; }
}
echo "start $(date)" > "$OUT/status.txt"
run switch 300 python -u -m pytest tests/test_gpu_gemm_switch.py -q -k "ws_stagger" --timeout 240 --timeout-method thread
tail -2 "$OUT/switch.out"
run ab_off 200 python tools/gemm_ab.py --only fwd256 --M 6000000
run ab_on 200 env HGIN_WS_STAGGER=1 python tools/gemm_ab.py --only fwd256 --M 6000000
cat "$OUT/ab_off.out" "$OUT/ab_on.out"
if [ "${BENCH:-1}" = "1" ]; then
  run bench_on 400 env HGIN_WS_STAGGER=1 python bench.py --steps 10 --warmup 3
  tail -c 400 "$OUT/bench_on.out"
fi
echo "done $(date)" >> "$OUT/status.txt"
