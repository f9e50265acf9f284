#!/bin/bash
# round 6: stem BN partial rows group-reduced in the stem conv (16 rows for the fused BN/pool pass) — tests, R34 x5
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/stemgrp
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q -k "stem or resnet34" --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3 4 5; do
  for t in on off; do
    v=1; [ $t = off ] && v=0
    KML_TMP_STEMGRP=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null || exit 1
    echo "r34 stemgrp $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
