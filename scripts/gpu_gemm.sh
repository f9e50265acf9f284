#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $out/gemm_tests.log 2>&1
rc=$?; tail -15 $out/gemm_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/gemm_bench.py --tokens 16384 --write $out/gemm_tuning.json > $out/gemm_bench.jsonl 2> $out/gemm_bench.err || { tail -20 $out/gemm_bench.err; exit 1; }
python -c "
import json
for l in open('$out/gemm_bench.jsonl'):
    d=json.loads(l)
    if 'summary' in d: print(d)
    else: print(d['shape'], d['layout'], d['M'], d['N'], d['K'], 'torch', d['torch_us'], d['torch_TF'], 'kml', d['best'], d['best_us'], d['best_TF'], d['speedup_vs_torch'])
"
