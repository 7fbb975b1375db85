#!/bin/bash
# SQ counters of the fp32 weight-stationary GEMMs at the cfg3 shapes (tools/gemm_ab.py, M = 3M rows): the forward
# k_ws_f32 / k_wsf_f32 (fwd256, HGIN_WS_PIPE = 0 / 1), the PReLU-fused dW k_wsd_f32 / k_wsp_f32 (dw256pro,
# HGIN_WSD_PIPE = 0 / 1).  One
# rocprofv3 --pmc pass per counter group, each in its own run under its own time limit.
#   OUT=gpurun_out/x bash tools/gpu_gemm_pmc2.sh
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/gemm_pmc2}; mkdir -p "$OUT"; export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
         "GRBM_GUI_ACTIVE GRBM_COUNT")
# shape:HGIN_WSD_PIPE:HGIN_WS_PIPE
for v in ${VARIANTS:-"fwd256:1:0" "fwd256:1:1" "dw256pro:0:0" "dw256pro:1:0"}; do
  IFS=: read -r shape wsd ws <<< "$v"
  i=0
  for C in "${GROUPS_[@]}"; do
    i=$((i+1))
    d="$OUT/${shape}_wsd${wsd}_ws${ws}_p$i"
    HGIN_WSD_PIPE=$wsd HGIN_WS_PIPE=$ws timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_ws" \
      --output-format csv -d "$d" -o run -- python3 tools/gemm_ab.py --only "$shape" --M 3000000 --reps 3 \
      > "$d.log" 2>&1 || { echo "FAIL $shape wsd$wsd ws$ws pass $i"; tail -5 "$d.log"; exit 1; }
  done
done
echo done > "$OUT/status.txt"
