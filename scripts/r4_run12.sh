#!/bin/bash
# fresh ResNet-50 and BERT numbers + kernel tables at HEAD
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_head.json 2> $out/r50_head.err || { tail -20 $out/r50_head.err; exit 1; }
tail -1 $out/r50_head.json
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_head.json 2> $out/bert_head.err || { tail -20 $out/bert_head.err; exit 1; }
tail -1 $out/bert_head.json
rm -rf $out/pr50 $out/pbert
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pr50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 8 > $out/pr50.log 2>&1 || { tail -20 $out/pr50.log; exit 1; }
db=$(find $out/pr50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 60 > $out/r50_prof.md
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r50_timeline.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pbert -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pbert.log 2>&1 || { tail -20 $out/pbert.log; exit 1; }
db=$(find $out/pbert -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 60 > $out/bert_prof.md
python tools/rocpd_timeline.py $db --first-kernel k_embed_fwd --nth -2 > $out/bert_timeline.md
rm -rf $out/pr50 $out/pbert
tail -2 $out/r50_timeline.md $out/bert_timeline.md
