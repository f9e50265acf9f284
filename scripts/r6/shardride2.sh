#!/bin/bash
# round 6: 1-rank --force-comm rehearsal, end-of-backward shard vs shard riders (alternating), timeline
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/shardride
mkdir -p $out
for rep in 1 2; do
  for plan in "peer:shard:fp32:1024" "peer:shardride:fp32:1024"; do
    tag=$(echo $plan | tr ':' '_')
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off --force-comm --comm-plan $plan > $out/b_${tag}_$rep.json 2> $out/b_${tag}_$rep.err || { tail -20 $out/b_${tag}_$rep.err; exit 1; }
    echo "plan=$plan rep=$rep $(python -c "import json;d=json.loads(open('$out/b_${tag}_$rep.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('comm_plan'))")"
  done
done
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off --force-comm --comm-plan peer:shardride:fp32:1024 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline_shardride.md
tail -1 $out/r34_timeline_shardride.md
rm -rf $out/prof
