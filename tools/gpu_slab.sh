#!/bin/bash
# One-launch slab reduction: digests + timings in both modes, the GPU suite, cfg2 / cfg5 bench lines.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-slab}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -20 "$OUT/$name.log"; exit $rc ;; esac
}
HGIN_SLAB_REDUCE=2pass step slab_2pass 200 python tools/slab_check.py
step slab_fused 200 python tools/slab_check.py
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_cfg2 400 python bench.py --no-cpu-baseline
HGIN_SLAB_REDUCE=2pass step bench_cfg2_2pass 400 python bench.py --no-cpu-baseline
step bench_cfg5 600 python bench.py --config cfg5 --no-cpu-baseline
echo done >> "$OUT/status.txt"
cat "$OUT/slab_2pass.log" "$OUT/slab_fused.log"; tail -2 "$OUT/pytest_gpu.log"
for b in bench_cfg2 bench_cfg2_2pass bench_cfg5; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" "$OUT/$b.log"; done
