#!/bin/bash
# F1 small-batch workload: tests, batch_bench for both schemas, and a kernel profile of the cfg1 schema.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/batches
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_store.py tests/test_gpu_readout_loss.py tests/test_gpu_kernels.py -x -q > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 300 python tools/batch_bench.py --schema cfg1 > "$OUT/bb_cfg1.json" 2>&1 || exit 1
timeout -k 10 300 python tools/batch_bench.py --schema w128 > "$OUT/bb_w128.json" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg1" -o run -- \
  python3 tools/batch_bench.py --schema cfg1 --steps 20 --warmup 3 > "$OUT/prof.log" 2>&1 || exit 1
