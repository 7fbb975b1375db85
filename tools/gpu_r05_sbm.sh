#!/bin/bash
# round 5: the MFMA readout — store / small-batch tests, the step's time and profile, the readout's stamps
set -o pipefail
TAG=${TAG:-r05w}
TAG=$TAG bash tools/gpu_r05_store.sh || exit 1
timeout -k 10 200 python -u tools/sb_stamps.py > gpurun_out/$TAG/stamps.txt 2>&1 || exit 1
head -16 gpurun_out/$TAG/stamps.txt
