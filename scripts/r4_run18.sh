#!/bin/bash
# oneshot restriction + stem raw barriers + LN bwd prefetch: tests and R50 / R34 / BERT benches
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem or parity or oneshot" > $out/r18_tests.log 2>&1 || { tail -30 $out/r18_tests.log; exit 1; }
tail -1 $out/r18_tests.log
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_gpu.py -x -q --timeout 120 --timeout-method thread > $out/r18_tr_tests.log 2>&1 || { tail -30 $out/r18_tr_tests.log; exit 1; }
tail -1 $out/r18_tr_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r18.json 2> $out/r50_r18.err || { tail -20 $out/r50_r18.err; exit 1; }
tail -1 $out/r50_r18.json
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r18.json 2> $out/bert_r18.err || { tail -20 $out/bert_r18.err; exit 1; }
tail -1 $out/bert_r18.json
timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --no-epoch --e2e off > $out/r34_r18.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$out/r34_r18.json'));print('r34', d['ms_per_step'])"
rm -rf $out/pr50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pr50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 8 > $out/pr50.log 2>&1 || { tail -20 $out/pr50.log; exit 1; }
db=$(find $out/pr50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/r50_prof4.md
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r50_timeline4.md
rm -rf $out/pr50
head -22 $out/r50_prof4.md
