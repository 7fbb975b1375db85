#!/bin/bash
# round 6 final tree, call A: the GPU suite + smoke (tools/gpu_final.sh EVID=0), then the 2-rank gloo rehearsal of
# bench.py's multi-rank path on the one GPU (tools/gpu_dist_rehearsal.sh)
set -u
cd "$(dirname "$0")/.."
EVID=0 TAG=${TAG:-r06_final_a} bash tools/gpu_final.sh || exit $?
TAG=${TAG:-r06_final_a} bash tools/gpu_dist_rehearsal.sh
rc=$?
tail -c 600 gpurun_out/${TAG:-r06_final_a}/bench_2rank_gloo.json
exit $rc
