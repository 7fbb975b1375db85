#!/bin/bash
# round 5: small-batch step checks + per-kernel profile (TAG names the gpurun_out subdirectory)
set -o pipefail
TAG=${TAG:-r05i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_smallbatch.py tests/test_gpu_store.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -u tools/sb_prof.py --steps 400 > $OUT/plain.out 2>&1 || exit 1
cat $OUT/plain.out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/sb_prof.py --steps 200 > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \; | head -12
