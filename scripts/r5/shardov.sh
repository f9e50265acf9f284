#!/bin/bash
# staged ZeRO-1 plan: packed-rank correctness, then the 1-rank rehearsal A/B (same box)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $out/shardov_tests.log 2>&1 || { grep -E "PASS|FAIL|Error" $out/shardov_tests.log | tail -30; tail -60 $out/shardov_tests.log; exit 1; }
grep -E "PASS|FAIL|SKIP" $out/shardov_tests.log | tail -10
run() {
  local label=$1; shift
  timeout -k 10 150 python -u bench.py --steps 100 --warmup 5 --no-epoch --e2e off "$@" > $out/reh_$label.json 2> $out/reh_$label.err || { tail -8 $out/reh_$label.err; return 1; }
  python -c "import json;d=json.loads(open('$out/reh_$label.json').read().strip().splitlines()[-1]);print('$label', d['ms_per_step'], d['config'].get('comm_plan'), d.get('allreduce_ms'))"
}
for rep in 1 2; do
run base$rep || exit 1
run shard$rep --force-comm --comm-plan peer:shard:fp32:1024 || exit 1
run ov64_$rep --force-comm --comm-plan peer:shardov:fp32:64 || exit 1
run ov16_$rep --force-comm --comm-plan peer:shardov:fp32:16 || exit 1
run ov256_$rep --force-comm --comm-plan peer:shardov:fp32:256 || exit 1
done
