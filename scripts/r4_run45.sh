#!/bin/bash
# BERT weight-gradient slab split-K: wider splits grid (up to 8x the one-tile-per-CU count)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 600 python tools/gemm_bench.py --rounds 3 --reps 5 --tiles 256x256x8,128x128x2 \
  --shapes "2:2304:768:16384;2:768:768:16384;2:3072:768:16384;2:768:3072:16384" > $out/wgrad_bert_sweep.log 2>&1 || { tail -5 $out/wgrad_bert_sweep.log; exit 1; }
grep '^{' $out/wgrad_bert_sweep.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l)
    if r.get('summary'): continue
    print(r['layout'], r['M'], r['N'], r['K'], 'best', r['best'], r['best_us'], 'torch', r['torch_us'])
"
