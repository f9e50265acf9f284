#!/bin/bash
# stem patch swizzle: tests, R50 + R34 bench, R50 profile (stem line)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem or parity or oneshot" > $out/stem_tests.log 2>&1 || { tail -30 $out/stem_tests.log; exit 1; }
tail -1 $out/stem_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_stem.json 2> $out/r50_stem.err || { tail -20 $out/r50_stem.err; exit 1; }
tail -1 $out/r50_stem.json
timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --no-epoch --e2e off > $out/r34_stem.json 2>/dev/null || exit 1
tail -1 $out/r34_stem.json
rm -rf $out/pr50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pr50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 8 > $out/pr50.log 2>&1 || { tail -20 $out/pr50.log; exit 1; }
db=$(find $out/pr50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/r50_prof3.md
rm -rf $out/pr50
head -24 $out/r50_prof3.md
