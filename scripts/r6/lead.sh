#!/bin/bash
# round 6: rider blocks leading vs trailing the conv-pair grid (headline SGD riders; shard riders)
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/lead
mkdir -p $out
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardride > $out/p2.log 2>&1 || { tail -30 $out/p2.log; exit 1; }
grep " rel " $out/p2.log
for rep in 1 2; do
  for v in local:none local:all ride:zs ride:none; do
    kind=${v%%:*}; lead=${v##*:}
    args="--steps 100 --warmup 10 --no-epoch --e2e off"
    [ $kind = ride ] && args="$args --force-comm --comm-plan peer:shardride:fp32:1024"
    KUBEML_COMM_RIDE_HOSTS=a KUBEML_RIDER_LEAD=$lead timeout -k 10 200 python -u bench.py $args > $out/b_${kind}_${lead}_$rep.json 2> $out/b_${kind}_${lead}_$rep.err || { tail -20 $out/b_${kind}_${lead}_$rep.err; exit 1; }
    echo "v=$v rep=$rep $(tail -1 $out/b_${kind}_${lead}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
  done
done
