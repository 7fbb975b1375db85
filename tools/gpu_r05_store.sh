#!/bin/bash
# round 5: collation from coherent host descriptors — store / small-batch / boundary tests, then the step profile
set -o pipefail
OUT=gpurun_out/${TAG:-r05q}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_store.py tests/test_gpu_smallbatch.py tests/test_gpu_model.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/sb_prof.py --steps 400 > $OUT/plain.out 2>&1 || exit 1
cat $OUT/plain.out
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/sb_prof.py --steps 200 > $OUT/prof.log 2>&1 || exit 1
