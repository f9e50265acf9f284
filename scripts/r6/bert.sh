#!/bin/bash
# round 6: BERT on hand-written GEMMs only — tests, step bench, kernel table + timeline
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6/bert
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py \
  tests/test_bert_gpu.py tests/test_transformer_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/bench_bert.py --steps 30 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.json | cut -c1-400
cd /tmp && cd $R
rm -rf $out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python tools/bench_bert.py --steps 5 --warmup 2 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 7 --top 40 > $out/bert_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_mlm_mask --nth -2 > $out/bert_timeline.md
head -30 $out/bert_summary.md
tail -1 $out/bert_timeline.md
rm -rf $out/prof
