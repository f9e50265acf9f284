#!/bin/bash
# round 6: GPU suite, then shard vs shardride (same box, alternating) for the plan probe
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
bash scripts/r6/suite.sh suite6 || exit 1
out=$GRAFT_REPO_ROOT/gpurun_out/r6/ridefinal
mkdir -p $out
for rep in 1 2 3; do
  for plan in "peer:shard:fp32:1024" "peer:shardride:fp32:1024"; do
    tag=$(echo $plan | tr ':' '_')
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off --force-comm --comm-plan $plan > $out/b_${tag}_$rep.json 2> $out/b_${tag}_$rep.err || { tail -20 $out/b_${tag}_$rep.err; exit 1; }
    echo "plan=$plan rep=$rep $(tail -1 $out/b_${tag}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
  done
done
