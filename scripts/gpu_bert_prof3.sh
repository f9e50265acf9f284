#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/pb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pb -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pb.log 2>&1 || { tail -20 $out/pb.log; exit 1; }
db=$(find $out/pb -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 5 --top 45 > $out/bert_prof.md
python tools/rocpd_timeline.py $db --first-kernel k_embed_fwd --nth -2 > $out/bert_timeline.md
rm -rf $out/pb
head -60 $out/bert_prof.md
tail -2 $out/bert_timeline.md
