#!/bin/bash
# HEAD check: whole GPU suite, driver smoke, headline bench.
set -o pipefail
out=gpurun_out/head
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 200 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
