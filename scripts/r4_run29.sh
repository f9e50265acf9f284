#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $out/r29_tests.log 2>&1 || { tail -30 $out/r29_tests.log; exit 1; }
tail -1 $out/r29_tests.log
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r29_$i.json 2> $out/bert_r29.err || { tail -20 $out/bert_r29.err; exit 1; }
python -c "import json;d=json.load(open('$out/bert_r29_$i.json'));print('bert', d['value'], d['ms_per_step'])"
done
rm -rf $out/pbert
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pbert -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pbert.log 2>&1 || { tail -20 $out/pbert.log; exit 1; }
db=$(find $out/pbert -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/bert_prof4.md
python tools/rocpd_timeline.py $db --first-kernel k_embed_fwd --nth -2 > $out/bert_timeline4.md
rm -rf $out/pbert
tail -1 $out/bert_timeline4.md
grep -c "at::native" $out/bert_timeline4.md || true
