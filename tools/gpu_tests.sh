#!/bin/bash
# Run a selection of GPU tests on the box: TESTS (paths / node ids) and K (a -k expression), one pytest process
# under its own time limit; output in gpurun_out/$TAG/.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread \
  ${K:+-k "$K"} ${EXTRA:-} > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc $rc" | tee "$OUT/status.txt"
tail -30 "$OUT/pytest.log"
exit $rc
