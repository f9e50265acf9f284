#!/bin/bash
# round 6: BERT step after the LDS work vs _abbase (alternating), kernel table of the new tree
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6/bertab
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_bert_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for t in new base; do
    root=$R; [ $t = base ] && root=$R/_abbase
    (cd $root && timeout -k 10 300 python -u tools/bench_bert.py --steps 30 --warmup 5 > $out/b_${t}_$rep.json 2> $out/b_${t}_$rep.err) || { tail -20 $out/b_${t}_$rep.err; exit 1; }
    echo "bert $t $rep $(tail -1 $out/b_${t}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d.get('ms_per_step'), d.get('value'))")"
  done
done
cd /tmp && cd $R
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python tools/bench_bert.py --steps 5 --warmup 2 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 7 --top 40 > $out/bert_summary.md
head -16 $out/bert_summary.md
rm -rf $out/prof
