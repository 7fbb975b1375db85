#!/bin/bash
# round 6: bf16 GEMM A/B at the cfg5 shapes (M = 3M rows) — the PReLU-fused dW (HGIN_WSD_PIPE 0 = k_wsd_bf16,
# 1 = k_wsp_bf16 staggered, 2 = unstaggered), the forward / dX weight-stationary kernels at 32 or 64 W columns per wave
# (HGIN_WS_CPW) — SQ counters of the dW variants, then the small-batch suite
set -o pipefail
TAG=${TAG:-r06c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do
  for P in 0 1 2; do
    HGIN_WSD_PIPE=$P timeout -k 10 120 python -u tools/gemm_ab.py --dtype bf16 --M 3000000 --reps 10 --only dw256pro,dw512 >> $OUT/ab_dw.txt 2>&1 || exit 1
  done
  for C in 32 64; do
    HGIN_WS_CPW=$C timeout -k 10 120 python -u tools/gemm_ab.py --dtype bf16 --M 3000000 --reps 10 --only fwd256,fwd256acc,dx256 >> $OUT/ab_fwd.txt 2>&1 || exit 1
  done
done
grep '^{' $OUT/ab_dw.txt $OUT/ab_fwd.txt | python3 -c "
import json,sys
for l in sys.stdin:
    f,j=l.split(':',1); d=json.loads(j)
    print(d['env'], {k:(v['ms'],v['GB_s'],v['kernels']) for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
G3="GRBM_GUI_ACTIVE GRBM_COUNT"
G4="FETCH_SIZE"
G5="WRITE_SIZE"
for P in 0 1; do
  i=0
  for C in "$G1" "$G2" "$G3" "$G4" "$G5"; do
    i=$((i+1))
    d="$OUT/pmc/dw256pro_pipe${P}_p$i"
    mkdir -p $OUT/pmc
    HGIN_WSD_PIPE=$P timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "k_ws" --output-format csv -d "$d" -o run -- \
      python3 tools/gemm_ab.py --dtype bf16 --only dw256pro --M 3000000 --reps 3 > "$d.log" 2>&1 || { echo "FAIL pmc $P $i"; tail -5 "$d.log"; exit 1; }
  done
done
python3 tools/sq_summary.py $OUT/pmc k_ws > $OUT/sq_summary.txt 2>&1; cat $OUT/sq_summary.txt | head -40
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_smallbatch.py > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
exit $rc
