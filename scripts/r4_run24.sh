#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u tools/bn_bw.py > $out/bn_bw.jsonl 2> $out/bn_bw.err || { tail -20 $out/bn_bw.err; exit 1; }
cat $out/bn_bw.jsonl
