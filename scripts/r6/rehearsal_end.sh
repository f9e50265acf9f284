#!/bin/bash
# round 6 end: 1-rank --force-comm rehearsal of the N > 1 step (peer kernels run, no link),
# shard vs shardride vs local, alternating x3 on one box
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/rehearsal_end
mkdir -p $out
for rep in 1 2 3; do
  for plan in "peer:shard:fp32:1024" "peer:shardride:fp32:1024"; do
    tag=$(echo $plan | tr ':' '_')
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off --force-comm --comm-plan $plan > $out/b_${tag}_$rep.json 2> $out/b_${tag}_$rep.err || { tail -20 $out/b_${tag}_$rep.err; exit 1; }
    echo "plan=$plan rep=$rep $(tail -1 $out/b_${tag}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
  done
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/b_local_$rep.json 2>/dev/null || exit 1
  echo "plan=local rep=$rep $(tail -1 $out/b_local_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
done
