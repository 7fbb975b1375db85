#!/bin/bash
# s21: SQ counters of the weight-stationary dW, PReLU-fused vs plain (bf16 and fp32, M = 6M, N = K = 256).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s21}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
i=0
for DT in bf16 f32; do
  for V in pro plain; do
    i=$((i+1))
    timeout -k 10 120 python3 tools/wsd_one.py $DT $V 6000000 >> "$OUT/times.txt" 2>&1 || { echo "FATAL time $DT $V"; exit 1; }
    timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-include-regex "k_wsd" --output-format csv -d "$OUT/p$i" -o run -- \
        python3 tools/wsd_one.py $DT $V 6000000 > "$OUT/p$i.out" 2> "$OUT/p$i.err"
    rc=$?; echo "p$i $DT $V rc=$rc" >> "$OUT/status.txt"
    [ $rc -eq 0 ] || { echo "FATAL p$i $rc"; tail -5 "$OUT/p$i.err"; exit $rc; }
  done
done
cat "$OUT/times.txt" | grep -v amdgpu
echo done >> "$OUT/status.txt"
