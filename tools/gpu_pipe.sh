#!/bin/bash
set -u
cd /root/repo
OUT=gpurun_out/pipe1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "aggregate or model" > $OUT/pytest.log 2>&1 || { echo "FATAL pytest $?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for P in 0 1; do
  HGIN_AGG_PIPE=$P timeout -k 10 300 python tools/agg_bench.py > $OUT/agg_f32_p$P.txt 2>&1 || { echo "FATAL agg f32 $P"; exit 1; }
  HGIN_AGG_PIPE=$P timeout -k 10 300 python tools/agg_bench.py --bf16 > $OUT/agg_bf16_p$P.txt 2>&1 || { echo "FATAL agg bf16 $P"; exit 1; }
done
cat $OUT/agg_*.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_cfg2.json 2>$OUT/bench_cfg2.err || { echo FATAL bench2; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --config cfg5 --steps 10 > $OUT/bench_cfg5.json 2>$OUT/bench_cfg5.err || { echo FATAL bench5; exit 1; }
cat $OUT/bench_cfg2.json $OUT/bench_cfg5.json | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'][:5], d['ms_per_step'], d['roofline']['frac'], d['mfma']['frac'])"
