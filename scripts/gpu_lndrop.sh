#!/bin/bash
# Hidden dropout fused into the LayerNorm kernels (BERT): tests + BERT bench A/B.
set -o pipefail
out=gpurun_out/lndrop
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_gpu.py -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  KUBEML_LN_DROP_FUSE=$v timeout -k 10 300 python tools/bench_bert.py --steps 20 > $out/bert_$v.json 2> $out/bert_$v.err || { tail -5 $out/bert_$v.err; exit 1; }
  echo "ln_drop_fuse=$v $(tail -1 $out/bert_$v.json | cut -c1-160)"
done
