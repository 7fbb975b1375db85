#!/bin/bash
# the fused small-batch step under rocprofv3 (per-kernel durations; TAG names the gpurun_out subdirectory)
set -o pipefail
OUT=gpurun_out/${TAG:-sbprof}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/sb_prof.py --steps 200 > $OUT/prof.log 2>&1 || exit 1
tail -2 $OUT/prof.log
