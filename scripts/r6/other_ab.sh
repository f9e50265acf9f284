#!/bin/bash
# round 6: ResNet-50 and BERT steps, this tree vs _abbase (HEAD of the round's first half), alternating x2
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/otherab
mkdir -p $out
for rep in 1 2; do
  for t in new base; do
    root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
    (cd $root && timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_${t}_$rep.log 2>&1) || { tail -20 $out/r50_${t}_$rep.log; exit 1; }
    echo "r50 $t $rep $(tail -1 $out/r50_${t}_$rep.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
for rep in 1 2; do
  for t in new base; do
    root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
    (cd $root && timeout -k 10 400 python -u tools/bench_bert.py > $out/bert_${t}_$rep.log 2>&1) || { tail -20 $out/bert_${t}_$rep.log; exit 1; }
    echo "bert $t $rep $(tail -1 $out/bert_${t}_$rep.log | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
