#!/bin/bash
set -o pipefail
out=gpurun_out/gb
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $out/gemm_tests.log 2>&1
rc=$?; tail -3 $out/gemm_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/gemm_bench.py --tokens 16384 --rounds 5 --reps 10 --tiles 256x256x8,256x256x4,128x128x2,128x128,256x128,128x256 --write $out/gemm_tuning.json > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l)
    if r.get('summary'): print(r); continue
    print(r['shape'], r['layout'], r['M'], r['N'], r['K'], 'torch', r['torch_us'], r['torch_TF'], '| best', r['best'], r['best_us'], r['best_TF'])
"
