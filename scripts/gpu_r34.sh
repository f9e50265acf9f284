#!/bin/bash
# Full GPU test suite, the headline bench (plain and single-rank graph-comm rehearsal), profile.
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --force-comm --graph-comm on 2>> $out/bench.err | tail -1 > $out/bench_gc.json || exit 1
cat $out/bench_gc.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 > $out/prof.log 2>&1 || exit 1
echo done
