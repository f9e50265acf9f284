#!/bin/bash
# round 6: 4x4 halo swizzle — halo tests, LDS-conflict PMC and kernel time
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/halo4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -k "halo or resnet34" --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/p2 $out/kt
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/p2 -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
python tools/pmc_table.py --steps 24 --top 40 $(find $out/p2 -name "*counter_collection.csv") | grep -E "kernel|halo<0, 128"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/kt.log 2>&1 || { tail -5 $out/kt.log; exit 1; }
db=$(find $out/kt -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/summary.md && grep -E "Per step|halo<0, 128" $out/summary.md
rm -rf $out/kt
