#!/bin/bash
# In-graph re-tune of the ResNet-34 backward plans with the round-3 forward kernels in place.
set -o pipefail
out=gpurun_out/tune3
mkdir -p $out
cp kubeml_amd/ops/conv_tuning.json $out/conv_tuning.json
timeout -k 10 1100 python -u tools/tune_ingraph.py --only bwd --topk 3 --out $out/conv_tuning.json > $out/tune.log 2>&1
rc=$?; tail -5 $out/tune.log; exit $rc
