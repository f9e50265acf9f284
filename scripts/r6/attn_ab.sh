#!/bin/bash
# round 6: attention backward specialised on dropout mode / bias (dKV at 3 waves per SIMD) vs _abbase
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6/attnab${1:-}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for t in new base; do
  root=$R; [ $t = base ] && root=$R/_abbase
  (cd $root && timeout -k 10 120 python -u tools/attn_micro.py > $out/micro_$t.log 2>&1) || { tail -20 $out/micro_$t.log; exit 1; }
  echo "== $t"; grep case $out/micro_$t.log
done
for rep in 1 2; do
  for t in new base; do
    root=$R; [ $t = base ] && root=$R/_abbase
    (cd $root && timeout -k 10 300 python -u tools/bench_bert.py --steps 30 --warmup 5 > $out/b_${t}_$rep.json 2> $out/b_${t}_$rep.err) || { tail -20 $out/b_${t}_$rep.err; exit 1; }
    echo "bert $t $rep $(tail -1 $out/b_${t}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d.get('ms_per_step'))")"
  done
done
cd /tmp && cd $R
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python tools/bench_bert.py --steps 5 --warmup 2 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 7 --top 40 > $out/bert_summary.md
grep attn $out/bert_summary.md
rm -rf $out/prof
