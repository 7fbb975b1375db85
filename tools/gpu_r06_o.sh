#!/bin/bash
# round 6: bf16 dW (PReLU-fused) and forward per-launch time against M (1M / 3M / 6M rows): where the in-step rate
# falls below the M = 3M A/B figures
set -u
OUT=gpurun_out/${TAG:-r06o}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for M in 1000000 3000000 6000000; do
  timeout -k 10 120 python -u tools/wsd_one.py bf16 pro $M >> "$OUT/wsd.log" 2>&1 || { tail -5 "$OUT/wsd.log"; exit 1; }
  timeout -k 10 120 python -u tools/gemm_ab.py --dtype bf16 --M $M --reps 10 --only fwd256,fwd256acc,dx256,dw256pro >> "$OUT/ab.log" 2>&1 || { tail -5 "$OUT/ab.log"; exit 1; }
done
cat "$OUT/wsd.log"
grep '^{' "$OUT/ab.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d['M'], {k:(v['ms'],v['GB_s']) for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
