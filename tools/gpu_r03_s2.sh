#!/bin/bash
# Round-3 checks: new kernel tests + variants + w256 + RCCL, then the aggregate LDS A/B on cfg3.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s2}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -40 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; }
}
run tests 900 python -u -m pytest ${TFILES:-tests/test_gpu_kernels.py tests/test_gpu_variants.py tests/test_gpu_model.py} \
    tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -rP \
    -k "${KSEL:-wsd_prelu or mlp_bwd_fused or global_pool or variant or w256 or rccl or global_feats}"
tail -3 "$OUT/tests.out"
run base 400 python bench.py --no-cpu-baseline --no-extras --steps 10
for D in ${DEPTHS:-8 16 24}; do
  HGIN_AGG_LDS=1 HGIN_AGG_LDS_D=$D run lds$D 400 python bench.py --no-cpu-baseline --no-extras --steps 10
done
for f in base $(for D in ${DEPTHS:-8 16 24}; do echo lds$D; done); do
  python3 -c "import json,sys; d=json.load(open('$OUT/$f.out')); r=d['roofline']; print('$f', d['ms_per_step'], r['achieved'], r['frac'], r['avg_launch_ms'])"
done
