#!/bin/bash
# Round 3: probe v2 (graph-branch vs eager side stream vs serial) + engine plan tests.
set -o pipefail
out=gpurun_out/r3comm2
mkdir -p $out
timeout -k 10 900 python -u tools/interference_probe.py --out $out/interference.json --plan-out $out/comm_plan.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep -v Warn $out/probe.log | tail -42
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "peer" > $out/engine_tests.log 2>&1
rc=$?; tail -8 $out/engine_tests.log; [ $rc = 0 ] || exit $rc
