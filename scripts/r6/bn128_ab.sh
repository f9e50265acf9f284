#!/bin/bash
# round 6: small single-batch BN applies on 128-thread blocks (twice the blocks) vs 256 — R34 x5
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bn128
mkdir -p $out
for rep in 1 2 3 4 5; do
  for t in on off; do
    if [ $t = on ]; then export KML_TMP_BN128=1; else unset KML_TMP_BN128; fi
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null || exit 1
    echo "r34 bn128 $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
