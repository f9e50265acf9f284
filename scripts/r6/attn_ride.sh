#!/bin/bash
# round 6: attention tests + dKV A/B (this tree vs the 429a6b7 tree), shardov bisect, shard riders
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/attn
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for t in new old; do
  root=$GRAFT_REPO_ROOT; [ $t = old ] && root=$GRAFT_REPO_ROOT/_bisect
  rm -rf /tmp/aprof_$t
  (cd $root && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/aprof_$t -o run -- python tools/attn_micro.py > $out/micro_$t.log 2>&1) || { tail -20 $out/micro_$t.log; exit 1; }
  f=$(find /tmp/aprof_$t -name "*kernel_stats.csv" | head -1)
  cp $f $out/kstats_$t.csv
  echo "== $t"; cat $out/micro_$t.log | grep -v Warn; grep "attn" $f | cut -d, -f1-5
done
bash scripts/r6/bis_ride.sh
