#!/bin/bash
# DGRAD row-pass epilogue: kernel tests, then ResNet-50 bench + per-call timing
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dgrad or conv_bwd_pair or conv_fwd_dgrad" > $out/rowpass_tests.log 2>&1 || { tail -30 $out/rowpass_tests.log; exit 1; }
tail -1 $out/rowpass_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_rowpass.json 2> $out/r50_rowpass.err || { tail -20 $out/r50_rowpass.err; exit 1; }
tail -1 $out/r50_rowpass.json
timeout -k 10 300 python -u tools/conv_calls.py --top 25 > $out/r50_calls2.txt 2> $out/r50_calls2.err || { tail -20 $out/r50_calls2.err; exit 1; }
grep "^#" $out/r50_calls2.txt | head -20
