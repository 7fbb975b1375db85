#!/bin/bash
# One GPU-box session: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / abort / timeout ends the script (no retries).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit status, $2 = step name
  case "$1" in
    0|1) return 0 ;;            # pass / ordinary test failure
    *) echo "FATAL: $2 exited $1; stopping" | tee -a "$OUT/status.txt"; exit "$1" ;;
  esac
}
echo "start $(date)" > "$OUT/status.txt"
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu $rc" >> "$OUT/status.txt"; stop_if_fatal $rc pytest
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench $rc" >> "$OUT/status.txt"; stop_if_fatal $rc bench
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof $rc" >> "$OUT/status.txt"; stop_if_fatal $rc rocprof
fi
echo "done $(date)" >> "$OUT/status.txt"
