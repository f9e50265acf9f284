#!/bin/bash
# stride-2 parity dgrad + 224 stem kernel: tests, then ResNet-50 bench + profile
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "parity or dgrad or conv_bwd_pair or stem" > $out/parity_tests.log 2>&1 || { tail -30 $out/parity_tests.log; exit 1; }
tail -1 $out/parity_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_parity.json 2> $out/r50_parity.err || { tail -20 $out/r50_parity.err; exit 1; }
tail -1 $out/r50_parity.json
rm -rf $out/pr50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pr50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 8 > $out/pr50.log 2>&1 || { tail -20 $out/pr50.log; exit 1; }
db=$(find $out/pr50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/r50_prof2.md
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r50_timeline2.md
rm -rf $out/pr50
tail -1 $out/r50_timeline2.md
