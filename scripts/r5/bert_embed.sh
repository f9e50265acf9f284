#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_gpu.py tests/test_bert_gpu.py > gpurun_out/r5/bert_embed_tests.log 2>&1 || { tail -30 gpurun_out/r5/bert_embed_tests.log; exit 1; }
tail -2 gpurun_out/r5/bert_embed_tests.log
for r in 1 2; do
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 3 > gpurun_out/r5/bert_embed_$r.json 2> gpurun_out/r5/bert_embed.err || { tail -20 gpurun_out/r5/bert_embed.err; exit 1; }
tail -1 gpurun_out/r5/bert_embed_$r.json | cut -c1-200
done
