#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
rm -rf $out/pbert
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pbert -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pbert.log 2>&1 || { tail -20 $out/pbert.log; exit 1; }
db=$(find $out/pbert -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/bert_prof3.md
python tools/rocpd_timeline.py $db --first-kernel k_embed_fwd --nth -2 > $out/bert_timeline3.md
rm -rf $out/pbert
tail -1 $out/bert_timeline3.md
