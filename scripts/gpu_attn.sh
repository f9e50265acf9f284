#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_gpu.py -x -q --timeout 150 --timeout-method thread > $out/attn_tests.log 2>&1
rc=$?; tail -3 $out/attn_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/bench_bert.py --steps 20 > $out/bert.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
cat $out/bert.json
