#!/bin/bash
# Look-ahead row kernel (HGIN_ROWS_PIPE): bit-identity, micro-bench and whole-step A/B on one box.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-rows_pipe}
mkdir -p "$OUT"
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  case $rc in 0) ;; *) echo "FATAL $name $rc"; tail -20 "$OUT/$name.log"; exit $rc ;; esac
}
step dig_base 200 python tools/rows_digest.py
HGIN_ROWS_PIPE=1 step dig_pipe 200 python tools/rows_digest.py
step rows_base 200 python tools/rows_bench.py
HGIN_ROWS_PIPE=1 step rows_pipe 200 python tools/rows_bench.py
step cfg5_base 600 python bench.py --config cfg5 --no-cpu-baseline
HGIN_ROWS_PIPE=1 step cfg5_pipe 600 python bench.py --config cfg5 --no-cpu-baseline
step cfg2_base 300 python bench.py --no-cpu-baseline
HGIN_ROWS_PIPE=1 step cfg2_pipe 300 python bench.py --no-cpu-baseline
timeout -k 10 300 python bench.py --config cfg2bf --no-cpu-baseline > "$OUT/bench_cfg2bf.json" 2>/dev/null
timeout -k 10 600 python bench.py --config cfg3 --no-cpu-baseline > "$OUT/bench_cfg3.json" 2>/dev/null
echo done >> "$OUT/status.txt"
grep -h "digest" "$OUT/dig_base.log" "$OUT/dig_pipe.log"
grep -hv amdgpu.ids "$OUT/rows_base.log" "$OUT/rows_pipe.log"
for b in cfg5_base cfg5_pipe cfg2_base cfg2_pipe; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" "$OUT/$b.log"; done
for c in cfg2bf cfg3; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline']['frac'])" "$OUT/bench_$c.json" || true; done
