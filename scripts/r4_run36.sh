#!/bin/bash
# ResNet-50: 1x1 weight gradients on gemm.hip's slab split-K (scripts/wgrad_gemm_r50.json) vs
# the implicit-GEMM wgrad, same box; BERT with the bias shadow in the library route
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "library or conv1x1" > $out/r36_tests.log 2>&1 || { tail -30 $out/r36_tests.log; exit 1; }
tail -1 $out/r36_tests.log
for i in 1 2; do
  unset KUBEML_WGRAD_GEMM_FILE
  timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r36_A_$i.json 2> $out/r50_r36.err || { tail -20 $out/r50_r36.err; exit 1; }
  echo "A $(tail -1 $out/r50_r36_A_$i.json | cut -c1-160)"
  export KUBEML_WGRAD_GEMM_FILE=scripts/wgrad_gemm_r50.json
  timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r36_B_$i.json 2> $out/r50_r36.err || { tail -20 $out/r50_r36.err; exit 1; }
  echo "B $(tail -1 $out/r50_r36_B_$i.json | cut -c1-160)"
done
unset KUBEML_WGRAD_GEMM_FILE
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r36.json 2> $out/bert_r36.err || { tail -20 $out/bert_r36.err; exit 1; }
echo "bert $(tail -1 $out/bert_r36.json | cut -c1-200)"
