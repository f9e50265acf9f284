#!/bin/bash
# BN folds (backward pair BNB + one-shot BN-in): numerics, then bench + per-dispatch timeline
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_bnb_gpu.py tests/test_models_gpu.py -x -v --timeout 120 --timeout-method thread > $out/fold1_tests.log 2>&1 || { tail -60 $out/fold1_tests.log; exit 1; }
grep -E "PASS|FAIL|SKIP" $out/fold1_tests.log | tail -20
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-epoch --e2e off > $out/fold1_bench.json 2> $out/fold1_bench.err || { tail -20 $out/fold1_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$out/fold1_bench.json').read().strip().splitlines()[-1]);print('ms', d['ms_per_step'], d['loss_first_last'])"
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/fold1_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/fold1_timeline.md
tail -3 $out/fold1_timeline.md
rm -rf $out/prof
