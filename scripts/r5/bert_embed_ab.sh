#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
for r in 1 2 3; do
  for f in 0 1; do
    KUBEML_EMBED_FUSED=$f timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 3 > gpurun_out/r5/bert_emb_${f}_$r.json 2> gpurun_out/r5/bert_emb.err || { tail -20 gpurun_out/r5/bert_emb.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/bert_emb_${f}_$r.json').read().strip().splitlines()[-1]);print('fused', $f, 'rep', $r, d['ms_per_step'])"
  done
done
