#!/bin/bash
# attention rework (XCD order, lazy rescale, stored dropout keep bits): tests, micro, BERT step
set -o pipefail
out=gpurun_out/attn2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_gpu.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for v in "1 4,2" "0 4,2" "1 3,3" "1 4,2"; do
  set -- $v
  KUBEML_ATTN_XCD=$1 KUBEML_ATTN_OCC=$2 timeout -k 10 120 python tools/attn_micro.py > $out/micro.jsonl 2>&1 || { cat $out/micro.jsonl; exit 1; }
  { echo "xcd=$1 occ=$2"; cat $out/micro.jsonl; } | tee -a $out/micro_all.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python tools/attn_micro.py > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 1 --top 12 > $out/attn_summary.md; rm -rf $out/prof
head -30 $out/attn_summary.md
timeout -k 10 300 python tools/bench_bert.py --steps 20 > $out/bert.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
cat $out/bert.json
