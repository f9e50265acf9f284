#!/bin/bash
# Round 3: peer transport tests, interference probe (-> comm plan), headline bench + rehearsals.
set -o pipefail
out=gpurun_out/r3comm
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_peer_gpu.py -x -v --timeout 200 --timeout-method thread > $out/peer_tests.log 2>&1
rc=$?; tail -5 $out/peer_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 600 python -u tools/interference_probe.py --out $out/interference.json --plan-out $out/comm_plan.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
tail -3 $out/probe.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "peer or rccl" > $out/engine_tests.log 2>&1
rc=$?; tail -5 $out/engine_tests.log; [ $rc = 0 ] || exit $rc
