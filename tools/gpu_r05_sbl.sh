set -o pipefail
TAG=${TAG:-r05m} bash tools/gpu_r05_sb.sh && mkdir -p gpurun_out/${TAG:-r05m} && timeout -k 10 200 python -u tools/sb_stamps.py > gpurun_out/${TAG:-r05m}/stamps.txt 2>&1; rc=$?; tail -30 gpurun_out/${TAG:-r05m}/stamps.txt; exit $rc
