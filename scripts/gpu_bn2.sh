#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/bn_latency.py > $out/bn_latency.log 2>&1 || { tail -5 $out/bn_latency.log; exit 1; }
cat $out/bn_latency.log
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
