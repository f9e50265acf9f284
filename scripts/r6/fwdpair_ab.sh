#!/bin/bash
# round 6: forward pairs of the downsampling blocks — tests, then ResNet-34 step vs _abbase (x4)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/fwdpair
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_fwd_pair_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3 4; do
  for t in new base; do
    root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
    (cd $root && timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null) || exit 1
    echo "r34 $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
