#!/bin/bash
# GEMM row-pass output epilogue: route tests, per-conv timings, ResNet-50 A/B (KUBEML_GEMM_OUT_ROWPASS=0 = old)
set -o pipefail
out=gpurun_out/r5/r50ab9; mkdir -p $out
KUBEML_GEMM_OUT_ROWPASS=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm_route or gather_route" --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
KUBEML_GEMM_OUT_ROWPASS=1 timeout -k 10 300 python -u tools/r50_1x1_micro.py --route > $out/route_new.txt 2>&1 || exit 1
KUBEML_GEMM_OUT_ROWPASS=0 timeout -k 10 300 python -u tools/r50_1x1_micro.py --route > $out/route_old.txt 2>&1 || exit 1
for v in new old new old; do
  if [ $v = old ]; then export KUBEML_GEMM_OUT_ROWPASS=0; else export KUBEML_GEMM_OUT_ROWPASS=1; fi
  timeout -k 10 300 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/r50_$v.json 2> $out/r50_$v.err || { tail -5 $out/r50_$v.err; exit 1; }
  echo "$v $(cat $out/r50_$v.json)" >> $out/ab.txt
done
