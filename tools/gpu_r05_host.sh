#!/bin/bash
# round 5: the small-batch step's host path — tests, host costs, the step's time
set -o pipefail
OUT=gpurun_out/${TAG:-r05s}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store.py tests/test_gpu_smallbatch.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/sb_host.py > $OUT/host.txt 2>&1 || { tail -20 $OUT/host.txt; exit 1; }
tail -1 $OUT/host.txt
timeout -k 10 120 python -u tools/sb_prof.py --steps 400 > $OUT/plain.out 2>&1 || exit 1
tail -1 $OUT/plain.out
