#!/bin/bash
# Round 4, third GPU call: full GPU suite (row-parallel small-batch step, pipelined dW default, the pipelined forward
# variant), smoke, the driver's bench command, the pipelined forward A/B (bench + per-shape), the batches profile and a
# kernel-trace summary of the cfg3 bench command.  Every GPU step time-limited; the script stops at the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04c}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc $(date +%T)" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -40 "$OUT/$name.out"; tail -30 "$OUT/$name.err"; exit $rc; }
}
echo "start $(date)" > "$OUT/status.txt"
if [ "${SUITE:-1}" = "1" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -2 "$OUT/pytest_gpu.out"
fi
run smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
tail -c 400 "$OUT/bench.out"
HGIN_WS_PIPE=1 run bench_ws_pipe 300 python bench.py --no-cpu-baseline --no-extras --no-probe --steps 10 --warmup 3
run bench_plain 300 python bench.py --no-cpu-baseline --no-extras --no-probe --steps 10 --warmup 3
grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_ws_pipe.out" "$OUT/bench_plain.out"
run gemm_ab_default 300 python tools/gemm_ab.py --only fwd256,dx256,dw256pro,dw512
run gemm_ab_wspipe 300 env HGIN_WS_PIPE=1 python tools/gemm_ab.py --only fwd256,dx256
cat "$OUT"/gemm_ab_*.out
run prof_batches 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_batches" -o run -- \
  python3 tools/batches_prof.py --steps 100
tail -c 600 "$OUT/prof_batches.out"
run prof_cfg3 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- \
  python3 bench.py --no-cpu-baseline --no-extras --no-probe --steps 5 --warmup 2
echo "done $(date)" >> "$OUT/status.txt"
