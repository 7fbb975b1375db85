#!/bin/bash
# Round-3 re-entry check: the 16-row PReLU-fused bf16 dW stages (targeted test first), the full GPU suite, smoke,
# cfg5 / cfg3 bench lines and the cfg5 kernel summary.  Each step time-limited; stop at the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s11}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -3 "$OUT/$name.out"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step wsd 300 python -u -m pytest tests/test_gpu_kernels.py -k "wsd or mlp_bwd" -x -q --timeout 120 --timeout-method thread
step suite 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_cfg5 400 python bench.py --config cfg5 --no-cpu-baseline
step bench_cfg3 400 python bench.py --no-cpu-baseline
step prof_cfg5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --config cfg5 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg5" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg5.txt"; head -12 "$OUT/summary_cfg5.txt"
step apl2 300 python tools/apl_bench.py
step apl3 300 env HGIN_APL_OCC=3 python tools/apl_bench.py
echo done >> "$OUT/status.txt"
