#!/bin/bash
# 256x192 phase tile: numerics vs fp32 torch, then the BERT-shape sweep vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r5/gemm_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/gemm_bench.py --tokens 16384 --rounds 5 --tiles 256x256x8,256x192x8 > gpurun_out/r5/gemm192_bench.jsonl 2> gpurun_out/r5/gemm192_bench.err
rc=$?
tail -3 gpurun_out/r5/gemm_tests.log
python - <<'PY'
import json
for l in open('gpurun_out/r5/gemm192_bench.jsonl'):
    d=json.loads(l)
    if d.get('summary'): print(d); continue
    a=d['all_us']; print(d['shape'], d['layout'], d['M'], d['N'], d['K'], 'torch', d['torch_us'], {k:v for k,v in a.items() if k!='torch'})
PY
exit $rc
