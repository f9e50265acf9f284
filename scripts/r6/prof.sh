#!/bin/bash
# round 6: default bench + per-dispatch ResNet-34 timeline (tag = $1)
set -o pipefail
export TMPDIR=/tmp
tag=${1:-base}
out=$GRAFT_REPO_ROOT/gpurun_out/r6/$tag
mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.json | cut -c1-300
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r34_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
tail -3 $out/r34_timeline.md
rm -rf $out/prof
