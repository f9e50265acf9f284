#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "kavg or gelu or conv1x1_wgrad" > $out/r35_kavg.log 2>&1 || { tail -30 $out/r35_kavg.log; exit 1; }
tail -1 $out/r35_kavg.log
timeout -k 10 120 python tools/diag/kavg_bits.py
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r35.json 2> $out/bert_r35.err || { tail -20 $out/bert_r35.err; exit 1; }
python -c "import json;d=json.load(open('$out/bert_r35.json'));print('bert', d['value'], d['ms_per_step'])"
rm -rf $out/pbert35
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pbert35 -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pbert35.log 2>&1 || { tail -20 $out/pbert35.log; exit 1; }
db=$(find $out/pbert35 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/bert_prof35.md
python tools/rocpd_timeline.py $db --first-kernel k_embed_fwd --nth -2 > $out/bert_timeline35.md
rm -rf $out/pbert35
tail -1 $out/bert_timeline35.md
timeout -k 10 300 python -u tools/wgrad_1x1.py > $out/wgrad_1x1.jsonl 2> $out/wgrad_1x1.err || { tail -20 $out/wgrad_1x1.err; exit 1; }
cat $out/wgrad_1x1.jsonl
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/r50_sync_comm.json 2> $out/r50_sync.err || { tail -20 $out/r50_sync.err; exit 1; }
python -c "import json;d=json.load(open('$out/r50_sync_comm.json'));print('r50 sync', d['value'], d['ms_per_step'], d.get('comm'), d.get('loss_first_last'))"
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm --async-kavg > $out/r50_async_comm.json 2> $out/r50_async.err || { tail -20 $out/r50_async.err; exit 1; }
python -c "import json;d=json.load(open('$out/r50_async_comm.json'));print('r50 async', d['value'], d['ms_per_step'], d.get('comm'), d.get('loss_first_last'))"
