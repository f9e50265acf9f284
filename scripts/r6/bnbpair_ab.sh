#!/bin/bash
# round 6: BN-backward apply pairs on / off (conv pairs on), alternating x5 on one box
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bnbpair
mkdir -p $out
for rep in 1 2 3 4 5; do
  for t in on off; do
    v=1; [ $t = off ] && v=0
    KUBEML_BWD_PAIR_AB=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null || exit 1
    echo "r34 bnbpair $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
