#!/bin/bash
# stride-2 parity dgrad: tests, then ResNet-50 bench + per-call timing
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "parity or dgrad or conv_bwd_pair" > $out/parity_tests.log 2>&1 || { tail -30 $out/parity_tests.log; exit 1; }
tail -1 $out/parity_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_parity.json 2> $out/r50_parity.err || { tail -20 $out/r50_parity.err; exit 1; }
tail -1 $out/r50_parity.json
timeout -k 10 300 python -u tools/conv_calls.py --top 25 > $out/r50_calls3.txt 2> $out/r50_calls3.err || { tail -20 $out/r50_calls3.err; exit 1; }
grep "^#" $out/r50_calls3.txt | head -24
