#!/bin/bash
# Quick GPU validation: gpu tests then the 1-GPU bench.
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -4 $out/gpu_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
