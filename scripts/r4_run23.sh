#!/bin/bash
# fused FFN GELU backward: BERT tests + bench + profile
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py tests/test_transformer_gpu.py tests/test_kernels_gpu.py -k "bert or attention or layernorm or ln or gelu or adam or sgd or optim" -x -q --timeout 120 --timeout-method thread > $out/r23_tests.log 2>&1 || { tail -30 $out/r23_tests.log; exit 1; }
tail -1 $out/r23_tests.log
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r23.json 2> $out/bert_r23.err || { tail -20 $out/bert_r23.err; exit 1; }
python -c "import json;d=json.load(open('$out/bert_r23.json'));print('bert', d['value'], d['ms_per_step'])"
rm -rf $out/pbert
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pbert -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pbert.log 2>&1 || { tail -20 $out/pbert.log; exit 1; }
db=$(find $out/pbert -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/bert_prof2.md
python tools/rocpd_timeline.py $db --first-kernel k_embed_fwd --nth -2 > $out/bert_timeline2.md
rm -rf $out/pbert
tail -1 $out/bert_timeline2.md
