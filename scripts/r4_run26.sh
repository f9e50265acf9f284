#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1; do
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r26_$i.json 2> $out/bert_r26.err || { tail -20 $out/bert_r26.err; exit 1; }
python -c "import json;d=json.load(open('$out/bert_r26_$i.json'));print('bert', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r26.json 2> $out/r50_r26.err || { tail -20 $out/r50_r26.err; exit 1; }
python -c "import json;d=json.load(open('$out/r50_r26.json'));print('r50', d['value'], d['ms_per_step'])"
timeout -k 10 200 python -u bench.py > $out/bench_default.json 2>/dev/null || exit 1
tail -1 $out/bench_default.json
