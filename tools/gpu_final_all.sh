#!/bin/bash
# Round-end evidence at HEAD: GPU suite + smoke, then tools/gpu_final_profiles.sh for cfg2 and cfg5.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/final_all
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/final_all/pytest_gpu.log 2>&1 || { echo "FATAL pytest $?"; tail -20 gpurun_out/final_all/pytest_gpu.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/final_all/smoke.log 2>&1 || { echo "FATAL smoke $?"; tail -20 gpurun_out/final_all/smoke.log; exit 1; }
CFG=cfg2 bash tools/gpu_final_profiles.sh && CFG=cfg5 bash tools/gpu_final_profiles.sh
rc=$?
tail -2 gpurun_out/final_all/pytest_gpu.log; tail -1 gpurun_out/final_all/smoke.log
tail -1 gpurun_out/final_cfg2/bench.out; tail -1 gpurun_out/final_cfg5/bench.out 2>/dev/null
exit $rc
