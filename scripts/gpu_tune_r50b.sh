#!/bin/bash
# Re-tune ResNet-50's conv plans (deterministic slab wgrad since round 2), then bench before/after.
set -o pipefail
out=gpurun_out/r50tune
mkdir -p $out
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/before.json 2> $out/before.err || { tail -5 $out/before.err; exit 1; }
tail -1 $out/before.json | cut -c1-200
cp kubeml_amd/ops/conv_tuning.json $out/conv_tuning.json
timeout -k 10 900 python -u tools/tune_conv.py --model resnet50 --batch 128 --size 224 --reps 5 --out $out/conv_tuning.json > $out/tune_r50.log 2>&1 || { tail -5 $out/tune_r50.log; exit 1; }
tail -3 $out/tune_r50.log
cp $out/conv_tuning.json kubeml_amd/ops/conv_tuning.json
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/after.json 2> $out/after.err || { tail -5 $out/after.err; exit 1; }
tail -1 $out/after.json | cut -c1-200
