#!/bin/bash
# same-box A/B: HEAD vs the tree of the first library-routing commit (ab_old/, 859c17e python
# + today's libraries) — checks nothing regressed BERT since the 16.76 ms box
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r43_new_$i.json 2> $out/bert_r43.err || { tail -20 $out/bert_r43.err; exit 1; }
  echo "new $(tail -1 $out/bert_r43_new_$i.json | cut -c60-130)"
  timeout -k 10 300 python -u ab_old/tools/bench_bert.py > $out/bert_r43_old_$i.json 2> $out/bert_r43.err || { tail -20 $out/bert_r43.err; exit 1; }
  echo "old $(tail -1 $out/bert_r43_old_$i.json | cut -c60-130)"
done
