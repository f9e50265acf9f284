#!/bin/bash
# round 6: rows per block of the BN-backward reduction pass (partial-row count) — R34 / R50 steps
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/rpb
mkdir -p $out
for rep in 1 2 3; do
  for m in 4 8 16; do
    KML_TMP_RPB=$m timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-epoch --e2e off > $out/r34_${m}_$rep.json 2>/dev/null || exit 1
    echo "r34 rpb$m $rep $(tail -1 $out/r34_${m}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for m in 4 8 16; do
    KML_TMP_RPB=$m timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_${m}_$rep.log 2>&1 || { tail -5 $out/r50_${m}_$rep.log; exit 1; }
    echo "r50 rpb$m $rep $(tail -1 $out/r50_${m}_$rep.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
