#!/bin/bash
# Kernel trace of the headline step at HEAD -> summary + one-step timeline.
set -o pipefail
out=gpurun_out/trace_now
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/r34
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/r34 -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/r34.log 2>&1 || { tail -20 $out/r34.log; exit 1; }
db=$(find $out/r34 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 50 > $out/r34_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
rm -rf $out/r34
tail -1 $out/r34_timeline.md
