#!/bin/bash
# Bias-as-ones-column wgrad: focused tests, bench, trace, then in-graph re-tune of the backward plans.
set -o pipefail
out=gpurun_out/r3perf2
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_peer_gpu.py -x -q --timeout 200 --timeout-method thread -k "determinism or bitwise or memset or one_update or first_update or overlap_matches or plans_on_one or unrolled or ce_bwd or conv or wgrad or linear or resnet or peer or gathered" > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cut -c1-300 $out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/r34
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/r34 -o run -- python bench.py --steps 20 --warmup 3 --no-epoch > $out/r34.log 2>&1 || { tail -20 $out/r34.log; exit 1; }
db=$(find $out/r34 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 45 > $out/r34_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
rm -rf $out/r34
tail -1 $out/r34_timeline.md
timeout -k 10 700 python -u tools/tune_ingraph.py --only bwd --topk 3 --out $out/conv_tuning.json > $out/tune.log 2>&1
rc=$?; tail -3 $out/tune.log; exit $rc
