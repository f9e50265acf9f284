#!/bin/bash
# round 6: maxpool backward row packing — pool / stem tests, then ResNet-34 vs _abbase-style HEAD build x3
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/poolab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "maxpool" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r34_summary.md
grep -E "maxpool|Per step" $out/r34_summary.md
rm -rf $out/prof
