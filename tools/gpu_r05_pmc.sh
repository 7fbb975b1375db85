#!/bin/bash
# Round 5: SQ counters of the fp32 weight-stationary GEMMs at the cfg3 shapes (tools/gemm_ab.py, M = 3M rows) —
# the PReLU-fused dW k_wsp_f32 (dw256pro: conflict-free slice reads), the dX-combine GEMM (dx256) and the
# accumulating forward (fwd256acc) under HGIN_WS_STAGGER = 1 / 0 (k_wss_f32 / k_ws_f32).  One rocprofv3 --pmc pass
# per counter group, each in its own run under its own time limit; tools/sq_summary.py reads them.
#   OUT=gpurun_out/x bash tools/gpu_r05_pmc.sh
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r05_pmc}; mkdir -p "$OUT"; export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
         "GRBM_GUI_ACTIVE GRBM_COUNT")
# shape:HGIN_WS_STAGGER
for v in ${VARIANTS:-"dw256pro:1" "dx256:1" "dx256:0" "fwd256acc:1" "fwd256acc:0"}; do
  IFS=: read -r shape st <<< "$v"
  i=0
  for C in "${GROUPS_[@]}"; do
    i=$((i+1))
    d="$OUT/${shape}_st${st}_p$i"
    HGIN_WS_STAGGER=$st timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_ws" \
      --output-format csv -d "$d" -o run -- python3 tools/gemm_ab.py --only "$shape" --M 3000000 --reps 3 \
      > "$d.log" 2>&1 || { echo "FAIL $shape st$st pass $i"; tail -5 "$d.log"; exit 1; }
  done
done
echo done > "$OUT/status.txt"
