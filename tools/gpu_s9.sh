#!/bin/bash
# Round-3 s9: B-DMA NT tile + split fused dW launch — parity (switch / variant / w256 tests), A/B timing, cfg3 bench
# and kernel profile.  Each step time-limited; stops at the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s9}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"; tail -4 "$OUT/$name.out"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
step tests 900 python -u -m pytest tests/test_gpu_gemm_switch.py tests/test_gpu_variants.py tests/test_gpu_h2.py \
    tests/test_gpu_model.py -x -q --timeout 400 --timeout-method thread \
    -k "switch or nt_bdma or nosums or f32_h2 or default or h2 or w256"
step ab_bdma_on 240 python tools/h2_bench.py
step ab_bdma_off 240 env HGIN_NT_BDMA=0 python tools/h2_bench.py
step bench_cfg3 600 python bench.py --config cfg3
step prof_cfg3 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
    python3 bench.py --config cfg3 --no-cpu-baseline --no-probe --no-extras
f=$(find "$OUT/prof_cfg3" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 23 > "$OUT/summary_cfg3.txt"
head -16 "$OUT/summary_cfg3.txt"
echo done >> "$OUT/status.txt"
