#!/bin/bash
# Round 3: deterministic gradients -> focused tests, bench, interference probe, whole GPU suite.
set -o pipefail
out=gpurun_out/r3det
mkdir -p $out
timeout -k 10 240 python -u -m pytest tests/test_determinism_gpu.py tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "determinism or bitwise or memset or one_update or first_update or overlap_matches or plans_on_one" > $out/det_tests.log 2>&1
rc=$?; tail -12 $out/det_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cut -c1-400 $out/bench.json
timeout -k 10 900 python -u tools/interference_probe.py --out $out/interference.json --plan-out $out/comm_plan.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep -v Warn $out/probe.log | tail -42
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -15 $out/gpu_tests.log; exit $rc
