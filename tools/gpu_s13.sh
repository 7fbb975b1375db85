#!/bin/bash
# SQ counter pass over the K = 512 fp32 forward GEMM: default k_gemm_nt (kBdma) vs the ping-pong k_nt_pp.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s13}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for PPV in 0 1; do
  for P in "$P1" "$P2"; do
    i=$((i+1))
    HGIN_NT_PP=$PPV timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "k_gemm|k_nt_pp" --output-format csv -d "$OUT/p$i" -o run -- \
        python3 tools/gemm_one.py fwd 3000000 512 256 > "$OUT/p$i.out" 2> "$OUT/p$i.err"
    rc=$?; echo "p$i pp=$PPV rc=$rc" >> "$OUT/status.txt"
    [ $rc -eq 0 ] || { echo "FATAL p$i $rc"; tail -5 "$OUT/p$i.err"; exit $rc; }
  done
done
echo done >> "$OUT/status.txt"
