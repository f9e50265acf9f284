#!/bin/bash
# round 6: full GPU suite + smoke + default bench (tag = $1)
set -o pipefail
export TMPDIR=/tmp
tag=${1:-suite}
out=$GRAFT_REPO_ROOT/gpurun_out/r6/$tag
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_suite.log 2>&1 || { tail -40 $out/gpu_suite.log; exit 1; }
tail -3 $out/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.json | cut -c1-200
