#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py tests/test_transformer_gpu.py tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread > $out/bert_tests.log 2>&1
rc=$?; tail -5 $out/bert_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/bench_bert.py --steps 10 > $out/bert.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
cat $out/bert.json
KUBEML_LINEAR_BLAS=1 timeout -k 10 300 python tools/bench_bert.py --steps 10 > $out/bert_blas.json 2> $out/bert_blas.err || { tail -20 $out/bert_blas.err; exit 1; }
cat $out/bert_blas.json
timeout -k 10 300 python tools/bench_bert.py --steps 10 --force-comm > $out/bert_fc.json 2> $out/bert_fc.err || { tail -20 $out/bert_fc.err; exit 1; }
cat $out/bert_fc.json
