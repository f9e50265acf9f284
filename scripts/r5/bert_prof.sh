#!/bin/bash
# current BERT-base step: kernel summary + per-dispatch timeline (copies, library GEMMs, attention)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r5
mkdir -p $out
rm -rf $out/prof_bert
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_bert -o run -- python tools/bench_bert.py --steps 5 --warmup 2 > $out/prof_bert.log 2>&1 || { tail -20 $out/prof_bert.log; exit 1; }
db=$(find $out/prof_bert -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 7 --top 30 > $out/bert_summary_r5.md && python tools/rocpd_timeline.py $db --first-kernel k_mlm_mask --nth -2 > $out/bert_timeline_r5.md
head -40 $out/bert_summary_r5.md
rm -rf $out/prof_bert
