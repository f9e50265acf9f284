#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 200 python tools/bn_latency.py > $out/bn_latency.log 2>&1 || { tail -5 $out/bn_latency.log; exit 1; }
cat $out/bn_latency.log
