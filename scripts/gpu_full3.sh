#!/bin/bash
# Full GPU suite + smoke + default bench (driver contract) at HEAD.
set -o pipefail
out=gpurun_out/full3
mkdir -p $out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/gputests.log 2>&1
rc=$?; tail -3 $out/gputests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cut -c1-2000 $out/bench.json
