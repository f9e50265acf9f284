#!/bin/bash
# XCD-aware attention block order: tests + graph-timed A/B on the BERT-base shape
set -o pipefail
out=gpurun_out/attn
mkdir -p $out
timeout -k 10 240 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for x in 0 1 0 1; do
  KUBEML_ATTN_XCD=$x timeout -k 10 120 python tools/attn_micro.py > $out/micro_xcd$x.jsonl 2>&1 || { cat $out/micro_xcd$x.jsonl; exit 1; }
  echo "xcd=$x"; cat $out/micro_xcd$x.jsonl
done
