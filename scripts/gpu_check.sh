#!/bin/bash
# GPU validation pass: new engine tests (verbose), the whole GPU suite, the 1-GPU bench
# (timed steps + measured epoch) and the 1-rank RCCL rehearsal of the overlapped step.
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 180 --timeout-method thread > $out/engine_tests.log 2>&1
rc=$?; tail -12 $out/engine_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -6 $out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 200 python bench.py --force-comm --overlap on --steps 100 --no-epoch > $out/bench_fc.json 2> $out/bench_fc.err || { tail -5 $out/bench_fc.err; exit 1; }
cat $out/bench_fc.json
