#!/bin/bash
# round 6: shard riders also on the BN-backward launches (thinner slices) vs conv launches only
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bnhost
mkdir -p $out
KUBEML_RIDE_BN_HOSTS=1 timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardride > $out/p2.log 2>&1 || { tail -30 $out/p2.log; exit 1; }
grep " rel " $out/p2.log
for rep in 1 2; do
  for v in 0 1; do
    KUBEML_RIDE_BN_HOSTS=$v timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off --force-comm --comm-plan peer:shardride:fp32:1024 > $out/b_${v}_$rep.json 2> $out/b_${v}_$rep.err || { tail -20 $out/b_${v}_$rep.err; exit 1; }
    echo "bnhosts=$v rep=$rep $(tail -1 $out/b_${v}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['config'].get('shard_riders'))")"
  done
done
