#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python tools/bench_resnet50.py > $out/r50.log 2>&1 || { tail -5 $out/r50.log; exit 1; }
tail -1 $out/r50.log
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
