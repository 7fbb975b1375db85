#!/bin/bash
# round 6: host-side fixes (folded Adam guards, masked BatchNorm, eval re-capture) + the staggered bf16 PRO dW
# (k_wsp_bf16) checked and A/B-timed against k_wsd_bf16<256,256,PRO> (HGIN_WSD_PIPE=0)
set -o pipefail
TAG=${TAG:-r06b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_kernels.py -k "wsd_prelu" > $OUT/pytest_k.log 2>&1 || { tail -30 $OUT/pytest_k.log; exit 1; }
tail -2 $OUT/pytest_k.log
for M in 3000000 6000000; do
  for P in 1 0; do
    HGIN_WSD_PIPE=$P timeout -k 10 120 python -u tools/wsd_one.py bf16 pro $M >> $OUT/ab.txt 2>&1 || exit 1
  done
done
cat $OUT/ab.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_smallbatch.py tests/test_gpu_model.py tests/test_gpu_bf16.py > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
exit $rc
