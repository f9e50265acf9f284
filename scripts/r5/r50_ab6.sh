#!/bin/bash
# ResNet-50 (224^2, batch 128) A/B: 3x3 weight gradients on the GEMM gather route (new) vs the implicit GEMM
set -o pipefail
out=gpurun_out/r5/r50ab6; mkdir -p $out
for v in new old new old; do
  if [ $v = old ]; then export KUBEML_WGRAD_GEMM_FILE=tools/diag/wgrad_gemm_r5_pre3x3.json; else unset KUBEML_WGRAD_GEMM_FILE; fi
  timeout -k 10 300 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/r50_$v.json 2> $out/r50_$v.err || { tail -5 $out/r50_$v.err; exit 1; }
  echo "$v $(cat $out/r50_$v.json)" >> $out/ab.txt
done
