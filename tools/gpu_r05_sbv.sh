#!/bin/bash
# The fused small-batch step per model switch (tools/sb_prof.py --model): ms per batch, then a rocprofv3 kernel
# summary of the MLP_BN + GLOBAL_FEATS variant.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-sbv}
mkdir -p "$OUT"
export TMPDIR=/tmp
for M in '{}' '{"global_feats": true, "bl_features": true}' '{"mlp_bn": true}' \
         '{"mlp_bn": true, "global_feats": true, "bl_features": true}' '{"node_embedding_size": 128}'; do
  timeout -k 10 200 python3 -u tools/sb_prof.py --steps 200 --model "$M" >> "$OUT/sbv.txt" 2>> "$OUT/sbv.err" || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bn" -o run -- \
    python3 tools/sb_prof.py --steps 200 --model '{"mlp_bn": true, "global_feats": true, "bl_features": true}' \
    > "$OUT/prof_bn.out" 2> "$OUT/prof_bn.err" || exit $?
f=$(find "$OUT/prof_bn" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" 20 > "$OUT/summary_bn.txt"
echo done >> "$OUT/sbv.txt"
