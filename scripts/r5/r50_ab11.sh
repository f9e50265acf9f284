#!/bin/bash
# ResNet-50: 28x28-output 3x3 weight gradients at 128 K-slices (new) vs 32 (old)
set -o pipefail
out=gpurun_out/r5/r50ab11; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad_gemm_gather" --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
for v in new old new old; do
  if [ $v = old ]; then export KUBEML_WGRAD_GEMM_FILE=tools/diag/wgrad_gemm_r5_split32.json; else unset KUBEML_WGRAD_GEMM_FILE; fi
  timeout -k 10 300 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/r50_$v.json 2> $out/r50_$v.err || { tail -5 $out/r50_$v.err; exit 1; }
  echo "$v $(cat $out/r50_$v.json)" >> $out/ab.txt
done
