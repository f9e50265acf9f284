#!/bin/bash
# Stem halo + BN fold: in-graph A/Bs.
set -o pipefail
out=gpurun_out/fold
mkdir -p $out
for cfg in "1 1 0" "1 1 1" "1 0 0" "0 0 0" "1 1 0" "1 1 1" "1 0 0" "0 0 0"; do
  set -- $cfg
  KUBEML_CONV_STEM=$1 KUBEML_BN_FOLD=$2 KUBEML_BN_FOLD_GROUP=$3 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "stem=$1 fold=$2 group=$3 $(python -c "import json;d=json.load(open('$out/ab.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
