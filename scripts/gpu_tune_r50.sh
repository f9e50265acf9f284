#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
cp kubeml_amd/ops/conv_tuning.json $out/conv_tuning.json
timeout -k 10 1000 python -u tools/tune_conv.py --model resnet50 --batch 128 --size 224 --reps 7 --out $out/conv_tuning.json > $out/tune_r50.log 2>&1 || { tail -5 $out/tune_r50.log; exit 1; }
tail -5 $out/tune_r50.log
