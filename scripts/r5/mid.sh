#!/bin/bash
# round-5 mid-round check: GPU suite, smoke, default bench, per-dispatch r34 timeline
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_suite2.log 2>&1 || { tail -40 $out/gpu_suite2.log; exit 1; }
tail -3 $out/gpu_suite2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke2.log 2>&1 || { tail -20 $out/smoke2.log; exit 1; }
tail -1 $out/smoke2.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_default3.json 2> $out/bench_default3.err || { tail -20 $out/bench_default3.err; exit 1; }
tail -1 $out/bench_default3.json | cut -c1-400
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/prof2.log 2>&1 || { tail -20 $out/prof2.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r34_summary2.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline2.md
tail -3 $out/r34_timeline2.md
rm -rf $out/prof
