#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py tests/test_transformer_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $out/r27_tests.log 2>&1 || { tail -30 $out/r27_tests.log; exit 1; }
tail -1 $out/r27_tests.log
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r27_$i.json 2> $out/bert_r27.err || { tail -20 $out/bert_r27.err; exit 1; }
python -c "import json;d=json.load(open('$out/bert_r27_$i.json'));print('bert', d['value'], d['ms_per_step'], d.get('loss_first_last'))"
done
