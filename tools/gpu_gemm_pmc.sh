#!/bin/bash
# SQ counters for the split-mode fp32 GEMMs (SHAPE=MxKxN, default the cfg2 l->p shape) (one rocprofv3 --pmc pass per group).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-gemm_pmc}; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
         "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_gemm" --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/gemm_bench.py --quick --shapes=${SHAPE:-600000x256x128} > $OUT/p$i.log 2>&1 || { echo "FAIL pass $i"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done > $OUT/status.txt
