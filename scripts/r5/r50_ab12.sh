#!/bin/bash
# row-pass epilogue reads in conflict-free 16-lane phases (new) vs the plain order (old, KUBEML_GEMM_ROWPASS_SWZ=0)
set -o pipefail
out=gpurun_out/r5/r50ab12; mkdir -p $out
KUBEML_GEMM_ROWPASS_SWZ=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm_route or gather_route" --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
for v in new old new old; do
  if [ $v = old ]; then export KUBEML_GEMM_ROWPASS_SWZ=0; else export KUBEML_GEMM_ROWPASS_SWZ=1; fi
  timeout -k 10 300 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/r50_$v.json 2> $out/r50_$v.err || { tail -5 $out/r50_$v.err; exit 1; }
  echo "$v $(cat $out/r50_$v.json)" >> $out/ab.txt
done
