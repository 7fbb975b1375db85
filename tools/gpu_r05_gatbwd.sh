#!/bin/bash
# round 5: the GAT backward with coalesced edge indices, U = 4 vs 8 edges in flight (HGIN_GAT_BWD_U), + its tests
set -o pipefail
OUT=gpurun_out/${TAG:-r05gat}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gat.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for U in 4 8; do
  HGIN_GAT_BWD_U=$U timeout -k 10 300 python -u tools/extras_probe.py --only gat > $OUT/gat_u$U.json 2>&1 || { tail -20 $OUT/gat_u$U.json; exit 1; }
  tail -1 $OUT/gat_u$U.json | cut -c1-600
done
export TMPDIR=/tmp
HGIN_GAT_BWD_U=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/extras_probe.py --only gat > $OUT/prof.log 2>&1 || exit 1
