#!/bin/bash
# In-graph A/B of conv tuning tables (isolated tuner timings do not carry over to the step):
#   bash scripts/gpu_ab_tables.sh tableA.json tableB.json ...   (each run twice, interleaved)
set -o pipefail
out=gpurun_out/ab
mkdir -p $out
for rep in 1 2; do
  for t in "$@"; do
    n=$(basename $t .json)
    KUBEML_CONV_TUNING_FILE=$t timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-epoch > $out/$n.$rep.json 2> $out/$n.err || { tail -5 $out/$n.err; exit 1; }
    echo "$n $(python -c "import json;print(json.load(open('$out/$n.$rep.json'))['ms_per_step'])")"
  done
done
