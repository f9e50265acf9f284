#!/bin/bash
# Fused stem: targeted tests, whole GPU suite, bench.
set -o pipefail
out=gpurun_out/stem
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "maxpool or stem" -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_all.log 2>&1
rc=$?; tail -3 $out/gpu_all.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
