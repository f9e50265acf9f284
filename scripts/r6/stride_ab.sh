#!/bin/bash
# round 6: shard riders on every conv-backward launch vs every 2nd / 3rd (1-rank rehearsal, alternating)
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/stride
mkdir -p $out
for rep in 1 2; do
  for k in 1 2 3; do
    KUBEML_RIDE_HOST_STRIDE=$k timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off --force-comm --comm-plan peer:shardride:fp32:1024 > $out/b_${k}_$rep.json 2> $out/b_${k}_$rep.err || { tail -20 $out/b_${k}_$rep.err; exit 1; }
    echo "stride=$k rep=$rep $(tail -1 $out/b_${k}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['config'].get('shard_riders'))")"
  done
done
