#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 120 python tools/diag/kavg_bits.py
timeout -k 10 300 python -u tools/wgrad_1x1.py > $out/wgrad_1x1.jsonl 2> $out/wgrad_1x1.err || { tail -20 $out/wgrad_1x1.err; exit 1; }
cat $out/wgrad_1x1.jsonl
