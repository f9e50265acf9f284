#!/bin/bash
# ResNet-50 / BERT with the shipped GEMM routes: bench + rocprofv3 kernel tables
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r40.json 2> $out/r50_r40.err || { tail -20 $out/r50_r40.err; exit 1; }
echo "r50 $(tail -1 $out/r50_r40.json | cut -c1-160)"
rm -rf $out/pr50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pr50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 2 > $out/pr50.log 2>&1 || { tail -20 $out/pr50.log; exit 1; }
db=$(find $out/pr50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/r50_prof40.md
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -3 > $out/r50_timeline40.md
rm -rf $out/pr50
tail -1 $out/r50_timeline40.md
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r40.json 2> $out/bert_r40.err || { tail -20 $out/bert_r40.err; exit 1; }
echo "bert $(tail -1 $out/bert_r40.json | cut -c1-200)"
