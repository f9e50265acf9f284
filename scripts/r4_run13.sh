#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u tools/conv_calls.py --top 40 > $out/r50_calls.txt 2> $out/r50_calls.err || { tail -20 $out/r50_calls.err; exit 1; }
grep "^#" $out/r50_calls.txt
