#!/bin/bash
# round 6: (1) the fp32 K = 512 forward against a two-pass K = 256 weight-stationary probe (tools/gemm_ab.py
# fwd512two); (2) SQ counters of the fused HetroGAT step's kernels (where k_sb_gat_fwd / _bwd waves spend their cycles)
set -u
OUT=gpurun_out/${TAG:-r06h}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bf16.py -k "nan or gin_mlp_fwd" \
  > "$OUT/pytest_nan.log" 2>&1 || { grep -E "^E |FAILED" "$OUT/pytest_nan.log" | head -20; tail -3 "$OUT/pytest_nan.log"; exit 1; }
tail -1 "$OUT/pytest_nan.log"
for rep in 1 2; do
  timeout -k 10 180 python -u tools/gemm_ab.py --M 3000000 --reps 10 --only fwd512acc,fwd512,fwd512two >> "$OUT/ab_k512.txt" 2>&1 \
    || { tail -20 "$OUT/ab_k512.txt"; exit 1; }
done
grep '^{' "$OUT/ab_k512.txt"
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
         "GRBM_GUI_ACTIVE GRBM_COUNT")
i=0
for C in "${GROUPS_[@]}"; do
  i=$((i+1))
  d="$OUT/sq/gat_p$i"
  mkdir -p "$OUT/sq"
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_sb_" --output-format csv -d "$d" -o run -- \
    python3 tools/sb_prof.py --steps 50 --gat > "$d.log" 2>&1 || { echo "FAIL pass $i"; tail -5 "$d.log"; exit 1; }
done
python3 tools/sq_summary.py "$OUT/sq" k_sb_ > "$OUT/sq_gat.txt" && cat "$OUT/sq_gat.txt"
