#!/bin/bash
# Kernel-trace profile of the ResNet-50 (224x224, batch 128) training step.
set -o pipefail
out=gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/p50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 2 --K 8 > $out/p50.log 2>&1 || { tail -20 $out/p50.log; exit 1; }
db=$(find $out/p50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 10 --top 40 > $out/r50_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r50_timeline.md
head -50 $out/r50_summary.md
tail -3 $out/r50_timeline.md
rm -rf $out/p50
