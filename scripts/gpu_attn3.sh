#!/bin/bash
# forward with two 16-query sub-tiles per wave (KUBEML_ATTN_QW), dKV with two key sub-tiles
# (KUBEML_ATTN_OCC=4,1): correctness + A/B
set -o pipefail
out=gpurun_out/attn3
mkdir -p $out
for v in "1 4,2" "2 4,1" "3 4,2"; do
  set -- $v
  KUBEML_ATTN_QW=$1 KUBEML_ATTN_OCC=$2 timeout -k 10 240 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  echo "qw=$1 occ=$2 $(tail -1 $out/tests.log)"
done
for v in "1 4,2" "2 4,2" "3 4,2" "1 4,1" "1 4,2" "2 4,2" "3 4,2" "1 4,1"; do
  set -- $v
  KUBEML_ATTN_QW=$1 KUBEML_ATTN_OCC=$2 timeout -k 10 120 python tools/attn_micro.py > $out/micro.jsonl 2>&1 || { cat $out/micro.jsonl; exit 1; }
  { echo "qw=$1 occ=$2"; grep -v amdgpu.ids $out/micro.jsonl; } | tee -a $out/micro_all.txt
done
