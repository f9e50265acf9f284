#!/bin/bash
# round-5 end: GPU suite, smoke, default bench, per-dispatch ResNet-34 timeline, ResNet-50 bench
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5/final
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_suite.log 2>&1 || { tail -40 $out/gpu_suite.log; exit 1; }
tail -3 $out/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
tail -1 $out/bench_default.json | cut -c1-300
timeout -k 10 300 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/bench_r50.json 2> $out/bench_r50.err || { tail -5 $out/bench_r50.err; exit 1; }
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r34_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
tail -3 $out/r34_timeline.md
rm -rf $out/prof
