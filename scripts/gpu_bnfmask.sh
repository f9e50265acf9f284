#!/bin/bash
# dgrad epilogue applies the consumer BN's ReLU mask (BN backward never reads y): tests + benches.
set -o pipefail
out=gpurun_out/bnfmask
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $out/gpu_all.log 2>&1
rc=$?; tail -3 $out/gpu_all.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('r34', d['ms_per_step'], d['value'], d.get('epoch_time_s'))"
timeout -k 10 300 python tools/bench_resnet50.py > $out/r50.log 2>&1 || { tail -5 $out/r50.log; exit 1; }
tail -1 $out/r50.log
