#!/bin/bash
# Kernel-trace profile of the headline step + per-step timeline summary.
set -o pipefail
out=gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
echo "db: $db"
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r34_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
tail -3 $out/r34_timeline.md
rm -rf $out/prof
