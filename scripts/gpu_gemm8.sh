#!/bin/bash
# k_gemm8 numerics + BERT-shape GEMM bench against hipBLASLt and the older tiles.
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $out/gemm_tests.log 2>&1
rc=$?; tail -3 $out/gemm_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/gemm_bench.py --tokens 16384 --rounds 5 --reps 10 --tiles 256x256x8,256x256x4,128x128x2,128x128 --write $out/gemm_tuning.json > $out/gemm_bench.log 2>&1 || { tail -5 $out/gemm_bench.log; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/gemm_bench.log'):
    r=json.loads(l)
    if r.get('summary'): print(r); continue
    a=r['all_us']
    print(r['shape'], r['layout'], r['M'], r['N'], r['K'], 'torch', r['torch_us'], '8ph', a.get('256x256x8st/s1'), 'best', r['best'], r['best_us'], r['best_TF'])
PY
