#!/bin/bash
# BERT-base step at HEAD (closing number for profiles/bert_base_r3.md)
set -o pipefail
out=gpurun_out/berthead
mkdir -p $out
timeout -k 10 300 python tools/bench_bert.py --steps 20 > $out/bert.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
cat $out/bert.json
