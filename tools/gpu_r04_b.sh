#!/bin/bash
# Round 4: the fused small-batch step's parity tests and profile; SQ counter passes of the weight-stationary fp32 GEMMs;
# the 2-rank rehearsals of bench.py's N > 1 legs with the probe on (cfg3 -> the cfg4 component split, and cfg5), each
# rank logging its peak device memory; then the CPU baseline on the FULL cfg2 graph (bench.py --cpu-full cfg2, the box's
# host cores).  Every GPU step time-limited; the script stops at the first
# failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04b}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc $(date +%T)" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -30 "$OUT/$name.err"; exit $rc; }
}
echo "start $(date)" > "$OUT/status.txt"
if [ "${SB:-1}" = "1" ]; then   # the fused small-batch step: parity, then its profile
  run pytest_sb 300 python -u -m pytest tests/test_gpu_smallbatch.py tests/test_gpu_store.py -q --timeout 120 --timeout-method thread
  tail -2 "$OUT/pytest_sb.out"
  run prof_batches 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_batches" -o run -- \
    python3 tools/batches_prof.py --steps 100
  tail -c 700 "$OUT/prof_batches.out"
fi
if [ "${PMC:-1}" = "1" ]; then
  run gemm_pmc2 900 env OUT="$OUT/gemm_pmc2" bash tools/gpu_gemm_pmc2.sh
fi
if [ "${REHEARSE:-1}" = "1" ]; then
  export HGIN_DIST_BACKEND=gloo
  run rehearse_cfg3 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2
  tail -c 1500 "$OUT/rehearse_cfg3.out"
  run rehearse_cfg5 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --config cfg5
  tail -c 1500 "$OUT/rehearse_cfg5.out"
  unset HGIN_DIST_BACKEND
fi
if [ "${CPUFULL:-1}" = "1" ]; then
  run cpu_full_cfg2 1000 python bench.py --cpu-full cfg2
  cat "$OUT/cpu_full_cfg2.out"
fi
echo "done $(date)" >> "$OUT/status.txt"
