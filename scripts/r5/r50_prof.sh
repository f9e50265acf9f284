#!/bin/bash
# ResNet-50 (224^2, b128) kernel table + one-step timeline after the 1x1 GEMM routes
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5/r50prof
mkdir -p $out
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r50_kernels.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r50_timeline.md
tail -3 $out/r50_timeline.md
rm -rf $out/prof
