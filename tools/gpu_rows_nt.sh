#!/bin/bash
# Non-temporal operand loads in the PReLU / combine backward row kernels (HGIN_ROWS_NT): micro-bench and
# whole-step A/B on one box.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-rows_nt}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -20 "$OUT/$name.log"; exit $rc ;; esac
}
step rows_base 200 python tools/rows_bench.py
HGIN_ROWS_NT=1 step rows_nt 200 python tools/rows_bench.py
step cfg2_base 300 python bench.py --no-cpu-baseline
HGIN_ROWS_NT=1 step cfg2_nt 300 python bench.py --no-cpu-baseline
step cfg2_base_b 300 python bench.py --no-cpu-baseline
HGIN_ROWS_NT=1 step cfg2_nt_b 300 python bench.py --no-cpu-baseline
HGIN_ROWS_NT=1 step cfg5_nt 600 python bench.py --config cfg5 --no-cpu-baseline
step cfg5_base 600 python bench.py --config cfg5 --no-cpu-baseline
echo done >> "$OUT/status.txt"
grep -h "" "$OUT/rows_base.log" "$OUT/rows_nt.log" | grep -v amdgpu.ids
for b in cfg2_base cfg2_nt cfg2_base_b cfg2_nt_b cfg5_nt cfg5_base; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" "$OUT/$b.log"; done
