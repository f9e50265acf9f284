#!/bin/bash
# Round-3 baseline at HEAD: headline bench, 1-rank RCCL rehearsal, framework (e2e) path.
set -o pipefail
out=gpurun_out/r3base
mkdir -p $out
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 200 python bench.py --force-comm --steps 200 --no-epoch > $out/bench_fc.json 2> $out/bench_fc.err || { tail -5 $out/bench_fc.err; exit 1; }
cut -c1-200 $out/bench_fc.json
timeout -k 10 400 python tools/bench_e2e.py --epochs 4 --validate > $out/e2e.json 2> $out/e2e.err || { tail -20 $out/e2e.err; exit 1; }
tail -c 1500 $out/e2e.json
