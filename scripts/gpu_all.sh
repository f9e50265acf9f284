#!/bin/bash
# Full GPU validation + the three benchmarks (R34 headline, BERT, R50).
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 python tools/bench_bert.py --steps 20 > $out/bert.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
cat $out/bert.json
timeout -k 10 300 python tools/bench_resnet50.py > $out/r50.log 2>&1 || { tail -5 $out/r50.log; exit 1; }
tail -1 $out/r50.log
