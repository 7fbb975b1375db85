#!/bin/bash
# Round 4, first tree on the GPU: full GPU suite, the driver's bench command (cfg3 headline + extras.cfg5), a kernel
# profile of the reference's real loop (extras.batches workload, tools/batch_bench.py cfg1 schema), and the 2-rank
# rehearsals of the N > 1 legs with the probe on (cfg3 -> cfg4 split, and cfg5).  Every GPU step time-limited; the
# script stops at the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04a}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?; echo "$name $rc $(date +%T)" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || { echo "FATAL $name $rc"; tail -30 "$OUT/$name.out"; tail -30 "$OUT/$name.err"; exit $rc; }
}
echo "start $(date)" > "$OUT/status.txt"
if [ "${SUITE:-1}" = "1" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -2 "$OUT/pytest_gpu.out"; grep -q " failed" "$OUT/pytest_gpu.out" && { grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.out"; exit 1; }
fi
run smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
tail -c 600 "$OUT/bench.out"
HGIN_DW512=tiled run bench_dw512_tiled 300 python bench.py --no-cpu-baseline --no-extras --no-probe --steps 10 --warmup 3
run bench_dw512_wsd 300 python bench.py --no-cpu-baseline --no-extras --no-probe --steps 10 --warmup 3
HGIN_WSD_PIPE=1 run bench_wsd_pipe 300 python bench.py --no-cpu-baseline --no-extras --no-probe --steps 10 --warmup 3
HGIN_WSD_PIPE=1 HGIN_WS_PIPE=1 run bench_both_pipe 300 python bench.py --no-cpu-baseline --no-extras --no-probe --steps 10 --warmup 3
grep -o '"ms_per_step": [0-9.]*' "$OUT"/bench_dw512_*.out "$OUT"/bench_*pipe.out
run prof_batches 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_batches" -o run -- \
  python3 tools/batches_prof.py --steps 100
if [ "${GEMMAB:-1}" = "1" ]; then
  run gemm_ab_default 300 python tools/gemm_ab.py
  run gemm_ab_t256 300 env HGIN_NT_T256=1 python tools/gemm_ab.py --only fwd512,fwd512acc
  run gemm_ab_dwtiled 300 env HGIN_DW512=tiled python tools/gemm_ab.py --only dw512
  run gemm_ab_wsdpipe 300 env HGIN_WSD_PIPE=1 python tools/gemm_ab.py --only dw512,dw256pro
  run gemm_ab_wspipe 300 env HGIN_WS_PIPE=1 python tools/gemm_ab.py --only fwd256,dx256
  cat "$OUT"/gemm_ab_*.out
fi
if [ "${REHEARSE:-1}" = "1" ]; then
  export HGIN_DIST_BACKEND=gloo
  run rehearse_cfg3 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2
  run rehearse_cfg5 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --config cfg5
fi
echo "done $(date)" >> "$OUT/status.txt"
