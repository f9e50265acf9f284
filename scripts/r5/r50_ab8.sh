#!/bin/bash
# ResNet-50 (224^2, batch 128) A/B: wide dgrads on the GEMM route with the row-pass epilogue (new) vs the implicit GEMM
set -o pipefail
out=gpurun_out/r5/r50ab8; mkdir -p $out
for v in new old new old; do
  if [ $v = old ]; then export KUBEML_CONV_TUNING_FILE=tools/diag/conv_tuning_r5_prerowpass.json; else unset KUBEML_CONV_TUNING_FILE; fi
  timeout -k 10 300 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/r50_$v.json 2> $out/r50_$v.err || { tail -5 $out/r50_$v.err; exit 1; }
  echo "$v $(cat $out/r50_$v.json)" >> $out/ab.txt
done
