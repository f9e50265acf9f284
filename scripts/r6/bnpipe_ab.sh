#!/bin/bash
# round 6: software-pipelined BN apply loops vs HEAD (_abbase): BN tests, bandwidth, R50 / R34 steps
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bnpipe
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "bn or BN or batchnorm or resnet" --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for t in new base; do
  root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
  (cd $root && timeout -k 10 200 python -u tools/bn_bw.py > $out/bw_$t.log 2>&1) || { tail -20 $out/bw_$t.log; exit 1; }
  echo "== $t"; grep '"M"' $out/bw_$t.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['M'],d['C'],d['res'],'apply',d['apply_us'],d['apply_TBps'],'bwd',d['bwd_us'],d['bwd_TBps'],'copy',d['copy_TBps'])"
done
for rep in 1 2; do
  for t in new base; do
    root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
    (cd $root && timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_${t}_$rep.log 2>&1) || { tail -20 $out/r50_${t}_$rep.log; exit 1; }
    echo "r50 $t $rep $(tail -1 $out/r50_${t}_$rep.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
    (cd $root && timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null) || exit 1
    echo "r34 $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
